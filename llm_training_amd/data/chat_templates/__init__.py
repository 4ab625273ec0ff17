"""Chat templates with ``{% generation %}`` assistant spans (for ``return_assistant_tokens_mask``).

Reference: src/llm_training/data/chat_templates/__init__.py:24-37 — ``get_chat_template`` accepts a
template NAME (one of the files here), a PATH to a template file, or a literal template string.
"""
from __future__ import annotations

from pathlib import Path

_DIR = Path(__file__).resolve().parent
NAMES = sorted(p.stem for p in _DIR.glob("*.j2"))


def get_chat_template(name_or_path_or_template: str | None) -> str | None:
    s = name_or_path_or_template
    if s is None:
        return None
    f = _DIR / f"{s}.j2"
    if f.exists():
        return f.read_text()
    p = Path(s)
    if len(s) < 4096 and p.exists() and p.is_file():
        return p.read_text()
    return s


__all__ = ["get_chat_template", "NAMES"]
