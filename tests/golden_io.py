"""Loading of the committed golden fixtures (tests/golden/*.json)."""
import json
import os

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name + ".json")) as fh:
        return json.load(fh)


def cases():
    """KAT + fuzz cases: dicts with sam, args, status, files (reference outputs)."""
    return load("kat") + load("fuzz")
