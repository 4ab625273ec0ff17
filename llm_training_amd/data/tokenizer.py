"""``HFTokenizer`` factory (reference src/llm_training/lightning/cli/utils.py:7-22): AutoTokenizer from a
LOCAL path with optional pad token / padding side overrides."""
from __future__ import annotations


def HFTokenizer(path: str, pad_token: str | None = None, padding_side: str | None = None, **kwargs):
    from transformers import AutoTokenizer

    kwargs.setdefault("local_files_only", True)
    tok = AutoTokenizer.from_pretrained(path, **kwargs)
    if pad_token is not None:
        tok.pad_token = pad_token
    if padding_side is not None:
        tok.padding_side = padding_side
    return tok
