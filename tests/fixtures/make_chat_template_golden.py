"""Regenerate chat_template_golden.json: renders (text + assistant spans) of the REFERENCE templates
(/root/reference/src/llm_training/data/chat_templates/*.j2, read as data) over a conversation corpus
with tools, tool_calls, ipython / tool turns, built-in tools and generation prompts, rendered by
transformers' own chat-template renderer. Cases where the reference template raises are recorded as
errors and not compared.

    python tests/fixtures/make_chat_template_golden.py [reference_template_dir]
"""
import json
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
TOOLS = [{"type": "function", "function": {"name": "get_weather", "description": "Weather in a city",
          "parameters": {"type": "object", "properties": {"city": {"type": "string"}}, "required": ["city"]}}}]
CORPUS = {
    "plain": [{"role": "user", "content": "hello  "}, {"role": "assistant", "content": " fine thanks"}],
    "system_multi": [{"role": "system", "content": "be nice "}, {"role": "user", "content": "hi"},
                     {"role": "assistant", "content": "yes"}, {"role": "user", "content": "again"},
                     {"role": "assistant", "content": "no"}],
    "tool_call": [{"role": "system", "content": "S"}, {"role": "user", "content": "weather in Paris?"},
                  {"role": "assistant", "content": "", "tool_calls": [
                      {"type": "function", "function": {"name": "get_weather", "arguments": {"city": "Paris"}}}]},
                  {"role": "tool", "content": "sunny"}, {"role": "assistant", "content": "It is sunny."}],
    "ipython": [{"role": "user", "content": "run"}, {"role": "assistant", "content": "", "tool_calls": [
                    {"type": "function", "function": {"name": "brave_search", "arguments": {"query": "x"}}}]},
                {"role": "ipython", "content": "{\"result\": 1}"}, {"role": "assistant", "content": "done"}],
    "two_tool_calls": [{"role": "user", "content": "q"}, {"role": "assistant", "content": "let me check",
                        "tool_calls": [{"function": {"name": "a", "arguments": {"x": 1}}},
                                       {"function": {"name": "b", "arguments": {"y": "z"}}}]},
                       {"role": "tool", "content": "r1"}, {"role": "tool", "content": "r2"},
                       {"role": "assistant", "content": "ok"}],
}
VARIANTS = {
    "default": {},
    "tools": {"tools": TOOLS},
    "tools_in_system": {"tools": TOOLS, "tools_in_user_message": False},
    "builtin_tools": {"builtin_tools": ["brave_search", "wolfram_alpha"], "tools": TOOLS},
    "generation_prompt": {"add_generation_prompt": True},
    "date": {"date_string": "01 Jan 2025"},
}


def render(template: str, messages, kw):
    from transformers.utils.chat_template_utils import render_jinja_template
    kw = dict(kw)
    kw.setdefault("date_string", "26 Jul 2024")  # llama-3.2 would otherwise print today's date
    tools = kw.pop("tools", None)
    try:
        out, spans = render_jinja_template(conversations=[messages], chat_template=template, tools=tools,
                                           return_assistant_tokens_mask=True, bos_token="<s>", eos_token="</s>",
                                           **kw)
        return {"text": out[0], "spans": [list(s) for s in spans[0]]}
    except Exception as e:  # noqa: BLE001
        return {"error": type(e).__name__}


def main():
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference/src/llm_training/data/chat_templates")
    golden = {}
    for f in sorted(ref.glob("*.j2")):
        golden[f.stem] = {f"{c}/{v}": render(f.read_text(), CORPUS[c], VARIANTS[v]) for c in CORPUS for v in VARIANTS}
    (HERE / "chat_template_golden.json").write_text(json.dumps(golden, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
