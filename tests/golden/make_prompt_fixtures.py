#!/usr/bin/env python3
"""Generate tests/golden/prompts.json from the reference's OWN prompt
functions (run here, where /root/reference exists; never on the GPU box).

The reference scripts cannot be imported (module top level fetches a model by
name: scratch.py:26, scratch2.py:26), so the pure host-side functions are
AST-extracted from the source text and executed in isolation with a stub
token model (the synthetic tokenizer): mix_contexts_and_query /
mix_multitoken_contexts_and_query (scratch2.py:50-78), generate_shuffled_prompt(s)
(scratch2.py:200-225), assemble_end_list_tasks (scratch2.py:240-245) and
construct_context / construct_query (scratch.py:45-48).  Each is called under
``random.seed(s)``; the inputs and outputs are stored as data.  No reference
source text is written anywhere.

    python tests/golden/make_prompt_fixtures.py
"""
import ast
import json
import random
import sys
import typing
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "prompts.json"

WANT = {
    "scratch2.py": ["mix_contexts_and_query", "mix_multitoken_contexts_and_query", "generate_shuffled_prompt",
                    "generate_shuffled_prompts", "assemble_end_list_tasks"],
    "scratch.py": ["construct_context", "construct_query"],
}


class _Ids(list):
    def tolist(self):
        return [list(self)]


class StubModel:
    """The TransformerLens token API the extracted functions call."""

    def __init__(self, tok):
        self.tok = tok

    def to_single_token(self, s):
        ids = self.tok.encode(s)
        assert len(ids) == 1, s
        return ids[0]

    def to_tokens(self, s, prepend_bos=True):
        return _Ids(([0] if prepend_bos else []) + self.tok.encode(s))


def extract(fname, names):
    tree = ast.parse((REF / fname).read_text())
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in names]
    assert {d.name for d in defs} == set(names), (fname, [d.name for d in defs])
    return ast.Module(body=defs, type_ignores=[])


def load_reference_functions(model):
    ns = {"random": random, "List": typing.List, "Tuple": typing.Tuple, "Tensor": object, "Float": object,
          "HookedTransformer": object, "model": model}
    for fname, names in WANT.items():
        exec(compile(extract(fname, names), f"<reference {fname} (extracted)>", "exec"), ns)
    return ns


def main():
    import tvr_amd
    cases = []
    make_cases(tvr_amd.tokenizer.SyntheticTokenizer(512), None, cases)
    # the same functions on a real byte-level BPE vocabulary (tests/golden/make_tokenizer.py)
    make_cases(tvr_amd.tokenizer.HFTokenizer(str(Path(__file__).resolve().parent / "tokenizer.json")), "hf", cases)
    OUT.write_text(json.dumps({"generator": "tests/golden/make_prompt_fixtures.py", "vocab": 512,
                               "cases": cases}, indent=1) + "\n")
    print(f"wrote {len(cases)} cases to {OUT}")


def make_cases(tok, tok_name, cases):
    import tvr_amd
    model = StubModel(tok)
    ref = load_reference_functions(model)
    T = tvr_amd.tasks

    def case(fn, seed, args, kwargs, out):
        c = {"fn": fn, "seed": seed, "args": args, "kwargs": kwargs, "out": out}
        if tok_name:
            c["tokenizer"] = tok_name
        cases.append(c)

    for seed, task, k, sep in [(0, "letter_to_caps", 4, None), (1, "low_to_caps", 6, ","), (2, "fruit_to_color", 3, "|"),
                               (3, "following_number", 5, None), (4, "state_to_capital", 5, ",")]:
        pairs = list(T.ALL_TASKS[task])
        random.seed(seed)
        pool = pairs.copy()
        random.shuffle(pool)
        demos, q = pool[:k], pool[k][0]
        one = all(len(tok.encode(s)) == 1 for s in [x for p in demos for x in p] + [q, T.ARROW] + ([sep] if sep else []))
        if task in ("fruit_to_color", "state_to_capital") or not one:
            out = ref["mix_multitoken_contexts_and_query"](demos, q, T.ARROW, sep, model)
            case("mix_multitoken_contexts_and_query", seed, [demos, q, T.ARROW, sep], {}, out)
        else:
            out = ref["mix_contexts_and_query"](demos, q, T.ARROW, sep, model)
            case("mix_contexts_and_query", seed, [demos, q, T.ARROW, sep], {}, out)
    for seed, task, n, k, f, sep in [(10, "letter_to_caps", 12, 4, T.ARROW, None),
                                     (11, "state_to_capital", 6, 3, ":", ","),
                                     (12, "fruit_to_color", 5, 4, ":", None)]:
        random.seed(seed)
        prompts, answers = ref["generate_shuffled_prompts"](list(T.ALL_TASKS[task]), model, n, k, f, sep)
        case("generate_shuffled_prompts", seed, [task, n, k, f, sep], {}, [prompts, answers])
    random.seed(20)
    states = list(T.us_states)
    lists = ref["assemble_end_list_tasks"](states, 7, 5)
    case("assemble_end_list_tasks", 20, [7, 5, ","], {}, [lists, states])
    random.seed(21)
    lists = ref["assemble_end_list_tasks"](list(T.us_states), 4, 3, "|")
    case("assemble_end_list_tasks", 21, [4, 3, "|"], {}, [lists, None])
    case("construct_context", None, [["a", "A"], T.ARROW], {}, ref["construct_context"](("a", "A"), T.ARROW))
    case("construct_query", None, [["b", "B"], ":"], {}, list(ref["construct_query"](("b", "B"), ":")))


if __name__ == "__main__":
    main()
