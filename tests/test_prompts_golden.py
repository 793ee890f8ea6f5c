"""CPU: the product's prompt builders (and the oracle's restatements) against
fixtures produced by the reference's own functions
(tests/golden/make_prompt_fixtures.py), same seeds, same global-random order."""
import json
import random
from pathlib import Path

import pytest

import tvr_amd
from oracle import reference_experiments as R

FIX = json.loads((Path(__file__).parent / "golden" / "prompts.json").read_text())
T = tvr_amd.tasks


class TokModel(tvr_amd.tokenizer.TokenizerMixin):
    def __init__(self, tokenizer):
        self.tokenizer = tokenizer
        self.device = "cpu"


M = TokModel(tvr_amd.tokenizer.SyntheticTokenizer(FIX["vocab"]))
# the same reference functions on a byte-level BPE vocabulary (tests/golden/make_tokenizer.py)
MODELS = {None: M, "hf": TokModel(tvr_amd.tokenizer.HFTokenizer(Path(__file__).parent / "golden" / "tokenizer.json"))}


def cases(fn):
    return [c for c in FIX["cases"] if c["fn"] == fn]


def cid(c):
    return f"{c['fn']}-{c['seed']}-{c.get('tokenizer', 'synthetic')}"


def as_pairs(x):
    return [tuple(p) for p in x]


@pytest.mark.parametrize("c", cases("mix_contexts_and_query") + cases("mix_multitoken_contexts_and_query"), ids=cid)
def test_icl_layouts(c):
    M = MODELS[c.get("tokenizer")]
    demos, q, f, sep = c["args"]
    demos = as_pairs(demos)
    if c["fn"] == "mix_contexts_and_query":
        assert tvr_amd.prompts.icl_single_token(M, demos, q, f, sep) == c["out"]
        assert R.mix_contexts_and_query(demos, q, f, sep, M) == c["out"]
    else:
        assert tvr_amd.prompts.icl_multi_token(M, demos, q, f, sep) == c["out"]
        assert R.mix_multitoken_contexts_and_query(demos, q, f, sep, M) == c["out"]


@pytest.mark.parametrize("c", cases("generate_shuffled_prompts"), ids=cid)
def test_generate_shuffled_prompts(c):
    M = MODELS[c.get("tokenizer")]
    task, n, k, f, sep = c["args"]
    want_p, want_a = c["out"]
    random.seed(c["seed"])
    p, a = tvr_amd.generate_shuffled_prompts(list(T.ALL_TASKS[task]), M, n, k, f, sep)
    assert p == want_p and a == want_a
    random.seed(c["seed"])
    p, a = R.generate_shuffled_prompts(list(T.ALL_TASKS[task]), M, n, k, f, sep)
    assert p == want_p and a == want_a


@pytest.mark.parametrize("c", cases("assemble_end_list_tasks"), ids=cid)
def test_assemble_end_list_tasks(c):
    n, k, sep = c["args"]
    want, want_mutated = c["out"]
    for fn in (tvr_amd.assemble_end_list_tasks, R.assemble_end_list_tasks):
        random.seed(c["seed"])
        objs = list(T.us_states)
        assert [list(x) for x in fn(objs, n, k, sep)] == want
        if want_mutated is not None:
            assert objs == want_mutated  # in-place shuffle of the caller's list (App. B6)


def test_construct_helpers():
    c1, c2 = cases("construct_context")[0], cases("construct_query")[0]
    assert tvr_amd.prompts.construct_context(tuple(c1["args"][0]), c1["args"][1]) == c1["out"]
    assert list(tvr_amd.prompts.construct_query(tuple(c2["args"][0]), c2["args"][1])) == c2["out"]


def test_extraction_prompt_stream_matches_reference_loop():
    """generate_mean_activation's prompt stream (scratch2.py:87-95): the
    product builds all prompts up front with the same shuffle order."""
    random.seed(77)
    ours = tvr_amd.prompts.sample_icl_prompts(M, T.letter_to_caps, T.ARROW, ",", 20, 4)
    random.seed(77)
    pool = list(T.letter_to_caps)
    ref = []
    for _ in range(20):
        random.shuffle(pool)
        ref.append(R.mix_multitoken_contexts_and_query(pool[:4], pool[4][0], T.ARROW, ",", M))
    assert ours == ref


def test_tokenizer_round_trip_on_task_data():
    for pairs in T.ALL_TASKS.values():
        for x, y in pairs:
            for s in (x, y):
                assert M.to_string(M.tokenizer.encode(s)) == s
    assert M.to_single_token(T.ARROW) != M.to_single_token(":")
    with pytest.raises(AssertionError):
        M.to_single_token(" New Hampshire")
    assert M.to_tokens("a")[0].tolist()[0] == 0
