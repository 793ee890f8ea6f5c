#!/usr/bin/env python3
"""Build tests/golden/tokenizer.json: a small byte-level BPE tokenizer with
the GPT-NeoX tokenizer's structure (byte-level pre-tokenizer without a prefix
space, byte-level decoder, ``<|endoftext|>`` = id 0 = BOS/EOS), trained
offline with the HF ``tokenizers`` library on the reference's task strings.

No tokenizer file of Pythia exists offline, so this stands in
for it in the tests of ``HFTokenizer`` / ``to_tokens`` / ``to_single_token`` /
``to_string`` (the TransformerLens API the reference calls at
scratch2.py:51,64,142,182,209,298): multi-token items (" New Hampshire"),
single-token letters, and the "→" / ":" / "," / "|" function and separator
tokens behave as they do with a real BPE vocabulary.

    python tests/golden/make_tokenizer.py
"""
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))

VOCAB = 480  # fits the tiny test model's 512-row embedding


def corpus():
    import tvr_amd
    T = tvr_amd.tasks
    lines = []
    for pairs in T.ALL_TASKS.values():
        for x, y in pairs:
            for f in ("→", ":", " →"):
                lines.append(f"{x}{f}{y}")
            lines.append(f"{x},{y}|{x}")
    lines += ["".join(T.us_states), ",".join(T.us_states), "|".join(T.us_states)]
    return lines * 4


def main():
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=VOCAB, special_tokens=["<|endoftext|>"], show_progress=False,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(corpus(), trainer=trainer)
    assert tok.token_to_id("<|endoftext|>") == 0
    out = HERE / "tokenizer.json"
    tok.save(str(out))
    print(f"wrote {out}: vocab {tok.get_vocab_size()}")


if __name__ == "__main__":
    main()
