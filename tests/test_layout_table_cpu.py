"""The shipped GEMM layout table (llm_training_amd/tuning/gemm_layouts_gfx950.json, consumed by ops/fused.py
_layout): every entry names a layout candidate that the GEMM entry points of its kind actually offer, so a
table edit (round 6 re-timed entries under longer interleaved rounds) can never select a missing variant, and
every key parses as that kind's problem key."""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "llm_training_amd", "tuning", "gemm_layouts_gfx950.json")

# candidate names per problem kind (ops/fused.py mm_nt / mm_nn / wgrad_into, each with a /nosk twin when
# stream-K is allowed)
_VALID = {
    "fwd": r"nt(/nosk)?",
    "dgrad": r"(tn|nn)(/nosk)?",
    "dgrad_wt": r"(tn|nn)(/nosk)?",
    "wgrad_dyt": r"tn(/nosk)?",
    "wgrad": r"((nt|tt|nn|tn)(2|4)?(/nosk)?|hip(2|4)?)",
}
# key fields after the kind: M|N|K|ld...|(dtype)|streamK
_KEY = {
    "fwd": r"\d+\|\d+\|\d+\|\d+\|\d+\|(True|False)\|(True|False)",
    "dgrad": r"\d+\|\d+\|\d+\|\d+\|\d+\|(True|False)",
    "dgrad_wt": r"\d+\|\d+\|\d+\|\d+\|\d+\|(True|False)",
    "wgrad_dyt": r"\d+\|\d+\|\d+\|\d+\|(bfloat16|float32)\|(True|False)",
    "wgrad": r"\d+\|\d+\|\d+\|\d+\|\d+\|(bfloat16|float32)\|(True|False)",
}


def test_table_entries_name_offered_candidates():
    with open(TABLE) as f:
        doc = json.load(f)
    assert doc["arch"] == "gfx950" and doc["about"]
    layouts = doc["layouts"]
    assert len(layouts) >= 79
    for key, val in layouts.items():
        kind, rest = key.split("|", 1)
        assert kind in _VALID, key
        assert re.fullmatch(_KEY[kind], rest), key
        assert re.fullmatch(_VALID[kind], val), (key, val)
        if val.endswith("/nosk"):  # a non-stream-K twin is offered only when stream-K is allowed
            assert key.endswith("|True"), (key, val)


def test_table_loaded_only_on_its_arch(monkeypatch):
    """ops/fused.py loads the shipped table only on the architecture it was measured on (its `arch` field); on
    another GPU the layouts are timed on first sight instead (round-5 advice). No device (CPU) loads it."""
    from llm_training_amd.ops import fused as F_
    for arch, expect in (("gfx950", True), ("gfx942", False), (None, True)):
        monkeypatch.setattr(F_, "_device_arch", lambda a=arch: a)
        monkeypatch.setattr(F_, "_LAYOUT_TABLE", [None])
        assert bool(F_._layout_table()) == expect, arch
