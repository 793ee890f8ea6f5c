"""ICL task datasets used by the reference experiments (data only).

Restated from the literals in scratch.py:28-41 and scratch2.py:28-41,
248-259, 320-373: letter case maps, fruit → colour, number → next number,
the 50 US states and state → capital.
"""
from __future__ import annotations

from typing import List, Tuple

Pairs = List[Tuple[str, str]]

_LOWER = "abcdefghijklmnopqrstuvwxyz"

# scratch.py:28-31 / scratch2.py:28-31
low_to_caps: Pairs = [(ch, ch.upper()) for ch in _LOWER]
caps_to_low: Pairs = [(ch.upper(), ch) for ch in _LOWER]
letter_to_caps: Pairs = low_to_caps + [(ch.upper(), ch.upper()) for ch in _LOWER]
letter_to_low: Pairs = caps_to_low + [(ch, ch) for ch in _LOWER]

# scratch.py:33-40 (27 pairs)
_FRUIT = """apple red|banana yellow|orange orange|strawberry red|blueberry blue|kiwi green|
watermelon green|pineapple yellow|mango orange|peach orange|pear green|plum purple|cherry red|
raspberry red|blackberry black|cantaloupe orange|honeydew green|papaya orange|apricot orange|
nectarine orange|lemon yellow|lime green|grapefruit orange|coconut white|pomegranate red|
fig purple|date brown"""
fruit_to_color: Pairs = [tuple(item.split()) for item in _FRUIT.replace("\n", "").split("|")]

# scratch.py:41
_NUMBERS = ["one", "two", "three", "four", "five", "six", "seven", "eight", "nine", "ten"]
following_number: Pairs = list(zip(_NUMBERS[:-1], _NUMBERS[1:]))

# scratch2.py:248-259 (leading spaces are part of each item)
_STATE_CAPITAL = [
    ("Alabama", "Montgomery"), ("Alaska", "Juneau"), ("Arizona", "Phoenix"),
    ("Arkansas", "Little Rock"), ("California", "Sacramento"), ("Colorado", "Denver"),
    ("Connecticut", "Hartford"), ("Delaware", "Dover"), ("Florida", "Tallahassee"),
    ("Georgia", "Atlanta"), ("Hawaii", "Honolulu"), ("Idaho", "Boise"),
    ("Illinois", "Springfield"), ("Indiana", "Indianapolis"), ("Iowa", "Des Moines"),
    ("Kansas", "Topeka"), ("Kentucky", "Frankfort"), ("Louisiana", "Baton Rouge"),
    ("Maine", "Augusta"), ("Maryland", "Annapolis"), ("Massachusetts", "Boston"),
    ("Michigan", "Lansing"), ("Minnesota", "St. Paul"), ("Mississippi", "Jackson"),
    ("Missouri", "Jefferson City"), ("Montana", "Helena"), ("Nebraska", "Lincoln"),
    ("Nevada", "Carson City"), ("New Hampshire", "Concord"), ("New Jersey", "Trenton"),
    ("New Mexico", "Santa Fe"), ("New York", "Albany"), ("North Carolina", "Raleigh"),
    ("North Dakota", "Bismarck"), ("Ohio", "Columbus"), ("Oklahoma", "Oklahoma City"),
    ("Oregon", "Salem"), ("Pennsylvania", "Harrisburg"), ("Rhode Island", "Providence"),
    ("South Carolina", "Columbia"), ("South Dakota", "Pierre"), ("Tennessee", "Nashville"),
    ("Texas", "Austin"), ("Utah", "Salt Lake City"), ("Vermont", "Montpelier"),
    ("Virginia", "Richmond"), ("Washington", "Olympia"), ("West Virginia", "Charleston"),
    ("Wisconsin", "Madison"), ("Wyoming", "Cheyenne"),
]
us_states: List[str] = [" " + s for s, _ in _STATE_CAPITAL]
us_states_capitals = {" " + s: " " + c for s, c in _STATE_CAPITAL}
# scratch2.py:373
state_to_capital_task: Pairs = [(s, us_states_capitals[s]) for s in us_states]

ARROW = "→"  # scratch.py:44, scratch2.py:45

ALL_TASKS = {
    "low_to_caps": low_to_caps,
    "caps_to_low": caps_to_low,
    "letter_to_caps": letter_to_caps,
    "letter_to_low": letter_to_low,
    "fruit_to_color": fruit_to_color,
    "following_number": following_number,
    "state_to_capital": state_to_capital_task,
}

# Strings the prompt builders put between items (function / separator tokens).
FUNCTION_TOKENS = [ARROW, ":", ",", "|", ", ", " →"]


def synthetic_task(n_pairs: int, vocab: int, seed: int, lo: int = 1000) -> Pairs:
    """A synthetic single-token task over token-id strings "<|id|>" (SURVEY.md
    §8d: items ~ U[1, V) with fixed function/separator ids).  Deterministic."""
    import random as _random

    rng = _random.Random(seed)
    ids = rng.sample(range(lo, vocab), 2 * n_pairs)
    return [(f"<|{ids[2 * i]}|>", f"<|{ids[2 * i + 1]}|>") for i in range(n_pairs)]
