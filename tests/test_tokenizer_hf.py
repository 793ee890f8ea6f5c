"""CPU: ``HFTokenizer`` (a local byte-level BPE ``tokenizer.json``, the form
Pythia's tokenizer ships in) behind the TransformerLens token API the
reference calls:

* ``to_tokens(str)`` prepends BOS = 0 (scratch2.py:182, hard-coded at :53,121,142),
  ``prepend_bos=False`` does not (:64,142,209);
* ``to_single_token`` asserts a single token (:51; TL's assert);
* ``to_string`` decodes ids / tensors (:43,298), keeping special tokens;
* string prompts of the reference's CIE path (generate_shuffled_prompts,
  :200-225) tokenize identically through the product and the oracle.
The fixture vocabulary is built offline by tests/golden/make_tokenizer.py.
"""
import random
from pathlib import Path

import pytest
import torch

import tvr_amd
from oracle import reference_experiments as R

TOK = Path(__file__).parent / "golden" / "tokenizer.json"
T = tvr_amd.tasks


class TokModel(tvr_amd.tokenizer.TokenizerMixin):
    def __init__(self):
        self.tokenizer = tvr_amd.tokenizer.HFTokenizer(TOK)
        self.device = "cpu"


M = TokModel()


def test_to_tokens_bos():
    ids = M.to_tokens("a→A")
    assert ids.dtype == torch.long and ids.shape[0] == 1
    assert ids[0, 0].item() == 0 and ids[0, 1:].tolist() == M.tokenizer.encode("a→A")
    assert M.to_tokens("a→A", prepend_bos=False)[0].tolist() == M.tokenizer.encode("a→A")
    assert M.tokenizer.encode("<|endoftext|>") == [0]


def test_to_single_token():
    for s in ("a", "A", T.ARROW, ":", ",", "|", "apple", "red"):
        assert isinstance(M.to_single_token(s), int)
    for s in (" New Hampshire", " Montgomery", " St. Paul"):
        with pytest.raises(AssertionError):
            M.to_single_token(s)


def test_to_string_round_trip():
    for pairs in T.ALL_TASKS.values():
        for x, y in pairs:
            for s in (x, y, x + ":" + y, x + T.ARROW + y):
                ids = M.tokenizer.encode(s)
                assert M.to_string(ids) == s
                assert M.to_string(torch.tensor(ids)) == s
    assert M.to_string(0) == "<|endoftext|>"
    assert M.to_string(torch.tensor(M.to_single_token("a"))) == "a"


def test_string_prompts_through_product_and_oracle():
    random.seed(31)
    p1, a1 = tvr_amd.generate_shuffled_prompts(list(T.state_to_capital_task), M, 5, 3, ":", ",")
    random.seed(31)
    p2, a2 = R.generate_shuffled_prompts(list(T.state_to_capital_task), M, 5, 3, ":", ",")
    assert p1 == p2 and a1 == a2
    assert any(len(a) > 1 for a in a1)  # multi-token capitals: the first token is the target (B3)
    assert all(M.to_tokens(p)[0, 0].item() == 0 for p in p1)


def test_rejects_a_vocabulary_whose_bos_is_not_zero(tmp_path):
    from tokenizers import Tokenizer, models, pre_tokenizers
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.add_tokens(["x"])
    tok.add_special_tokens(["<|endoftext|>"])
    p = tmp_path / "t.json"
    tok.save(str(p))
    with pytest.raises(ValueError, match="BOS"):
        tvr_amd.tokenizer.HFTokenizer(p)
