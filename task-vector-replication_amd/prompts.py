"""Prompt builders (host side): the token layouts the reference feeds its
forwards, with the same global-``random`` call order so a seeded run builds
the same prompts as the reference (App. B4, B6).

Layouts
  single-token ICL  [BOS] (x f y [s])*k [s] q f        scratch2.py:50-62
  multi-token ICL   same, each item tokenised          scratch2.py:63-78
  corrupted prompt  "x f y' [s]"*k + "q f" (y' = shuffled demo answers),
                    answer = tokens(y_q)                scratch2.py:200-225
  end-of-list task  (",".join(k states), k-th state)    scratch2.py:240-245
"""
from __future__ import annotations

import random
from typing import List, Optional, Sequence, Tuple

Pairs = List[Tuple[str, str]]

BOS = 0  # hard-coded by the reference (scratch.py:52, scratch2.py:53,121,142)


def icl_single_token(model, demos: Pairs, query: str, function_token: str = "→",
                     separator: Optional[str] = None) -> List[int]:
    """``mix_contexts_and_query`` (scratch2.py:50-62): every item must be one
    token (TL ``to_single_token`` asserts)."""
    one = model.to_single_token
    f = one(function_token)
    tail = [one(separator)] if separator is not None else []
    out = [BOS]
    for x, y in demos:
        out.extend([one(x), f, one(y)])
        out.extend(tail)
    out.extend(tail)  # separator doubled before the query (App. B4)
    out.extend([one(query), f])
    return out


def icl_multi_token(model, demos: Pairs, query: str, function_token: str = "→",
                    separator: Optional[str] = None) -> List[int]:
    """``mix_multitoken_contexts_and_query`` (scratch2.py:63-78)."""
    enc = model.tokenizer.encode
    f = enc(function_token)
    tail = enc(separator) if separator is not None else []
    out = [BOS]
    for x, y in demos:
        out += enc(x) + f + enc(y) + tail
    return out + tail + enc(query) + f


def sample_icl_prompts(model, contexts: Pairs, function_token: str, separator: Optional[str],
                       num_contexts: int, len_contexts: int) -> List[List[int]]:
    """The prompt stream of ``generate_mean_activation`` (scratch2.py:82-95):
    one in-place shuffle of a private copy per prompt; the first
    ``len_contexts`` pairs are demos, the next one the query."""
    pool = list(contexts)
    prompts = []
    for _ in range(num_contexts):
        random.shuffle(pool)
        prompts.append(icl_multi_token(model, pool[:len_contexts], pool[len_contexts][0],
                                       function_token, separator))
    return prompts


def generate_shuffled_prompt(contexts: Pairs, model, function_token: str = ":",
                             seperator_token: Optional[str] = None) -> Tuple[str, List[int]]:
    """scratch2.py:200-211: answers of the demos permuted, the last pair is the
    query; returns (prompt string without BOS, token ids of the query answer)."""
    demos, (q, q_answer) = contexts[:-1], contexts[-1]
    answers = [y for _, y in demos]
    random.shuffle(answers)
    sep = seperator_token if seperator_token is not None else ""
    body = "".join(f"{x}{function_token}{y}{sep}" for (x, _), y in zip(demos, answers))
    return body + q + function_token, model.tokenizer.encode(q_answer)


def generate_shuffled_prompts(contexts: Pairs, model, num_prompts: int, prompt_length: int,
                              function_token: str = ":", seperator_token: Optional[str] = None
                              ) -> Tuple[List[str], List[List[int]]]:
    """scratch2.py:213-225."""
    if prompt_length >= len(contexts):
        raise ValueError("Prompt length must be less than the number of contexts")
    pool = list(contexts)
    prompts, answers = [], []
    for _ in range(num_prompts):
        random.shuffle(pool)
        p, a = generate_shuffled_prompt(pool[:prompt_length + 1], model, function_token, seperator_token)
        prompts.append(p)
        answers.append(a)
    return prompts, answers


def assemble_end_list_tasks(objects: List[str], num_lists: int, num_elements: int,
                            seperator: str = ",") -> Pairs:
    """scratch2.py:240-245: the caller's list is shuffled in place (App. B6)."""
    out = []
    for _ in range(num_lists):
        random.shuffle(objects)
        out.append((seperator.join(objects[:num_elements]), objects[num_elements - 1]))
    return out


def construct_context(pair: Tuple[str, str], function_token: str = "→") -> str:
    """scratch.py:45-46."""
    return pair[0] + function_token + pair[1]


def construct_query(pair: Tuple[str, str], function_token: str = "→") -> Tuple[str, str]:
    """scratch.py:47-48."""
    return pair[0] + function_token, pair[1]


def synthetic_cie_prompts(model, n_prompts: int, k_shot: int, seed: int, n_pairs: int = 52,
                          function_token: str = "→") -> Tuple[List[List[int]], List[int]]:
    """Seeded synthetic corrupted prompts with single-token items (SURVEY.md
    §8d C3: T = 1 + 3k + 2, BOS + k shuffled-answer demos + query + f).
    Returns token-id prompts and the first answer token of each."""
    from .tasks import synthetic_task
    pairs = synthetic_task(n_pairs, model.cfg.d_vocab, seed)
    rng = random.Random(seed + 1)
    f = model.to_single_token(function_token)
    one = model.to_single_token
    prompts, answers = [], []
    for _ in range(n_prompts):
        pick = rng.sample(pairs, k_shot + 1)
        demo_answers = [y for _, y in pick[:-1]]
        rng.shuffle(demo_answers)
        ids = [BOS]
        for (x, _), y in zip(pick[:-1], demo_answers):
            ids += [one(x), f, one(y)]
        ids += [one(pick[-1][0]), f]
        prompts.append(ids)
        answers.append(one(pick[-1][1]))
    return prompts, answers
