"""Helpers to read tests/golden/kat_reference.json (data transcribed from the reference's tests)."""
import json
import os

from oracle import trie_ref as R

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "golden", "kat_reference.json")) as f:
        return json.load(f)


def b(s):
    return s.encode()


def dec_word(s):
    return {"''": R.EMPTY, "'+'": R.PLUS, "'#'": R.HASH}.get(s, s.encode() if isinstance(s, str) else s)
