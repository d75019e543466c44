"""Prompt formatting from the GGUF file itself, as llama-server does it.

The reference's LLM pod is upstream ``llama-server`` (reference cluster-config/apps/llm/
deployment.yaml:61,76-84): it formats ``/v1/chat/completions`` requests with the Jinja chat template
the model file carries (``tokenizer.chat_template``) and tokenises with the pre-tokeniser the file
names (``tokenizer.ggml.pre``).  This module does the same for the in-tree engine:

* :class:`ChatFormatter` renders ``tokenizer.chat_template`` in a sandboxed Jinja environment with
  the variables and helpers chat templates expect (``messages``, ``add_generation_prompt``,
  ``bos_token``, ``eos_token``, ``tools``, ``raise_exception``, ``strftime_now``, ``tojson``), with
  ``trim_blocks`` / ``lstrip_blocks`` like the template authors' reference renderer.  A file
  without a template falls back to ChatML (Qwen2.5-Instruct's format, llama-server's fallback).
* :func:`pre_tokenizer_pattern` maps ``tokenizer.ggml.pre`` to the split regex; a pre-type the
  engine does not implement is refused at load with a clear error instead of silently producing
  different token ids.
"""
from __future__ import annotations

import datetime
import json
from typing import Any, Dict, List, Optional, Sequence

# ``tokenizer.ggml.pre`` → split regex (the byte-level BPE pre-tokenisers of llama.cpp's vocab
# loader that this engine implements)
QWEN2 = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}|"
         r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
LLAMA3 = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}|"
          r" ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
GPT2 = r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+"
PRE_TOKENIZERS = {"qwen2": QWEN2, "llama3": LLAMA3, "llama-bpe": LLAMA3, "gpt-2": GPT2,
                  "default": GPT2}


# Qwen2.5-Instruct's ``tokenizer.chat_template`` (as its GGUF conversions carry it, with tool calls):
# written into the synthetic GGUF files so the served prompt path is the same as with the real file.
QWEN25_TEMPLATE = (
    "{%- if tools %}\n"
    "    {{- '<|im_start|>system\\n' }}\n"
    "    {%- if messages[0]['role'] == 'system' %}\n"
    "        {{- messages[0]['content'] }}\n"
    "    {%- else %}\n"
    "        {{- 'You are Qwen, created by Alibaba Cloud. You are a helpful assistant.' }}\n"
    "    {%- endif %}\n"
    "    {{- \"\\n\\n# Tools\\n\\nYou may call one or more functions to assist with the user query.\\n\\n"
    "You are provided with function signatures within <tools></tools> XML tags:\\n<tools>\" }}\n"
    "    {%- for tool in tools %}\n"
    "        {{- \"\\n\" }}\n"
    "        {{- tool | tojson }}\n"
    "    {%- endfor %}\n"
    "    {{- \"\\n</tools>\\n\\nFor each function call, return a json object with function name and "
    "arguments within <tool_call></tool_call> XML tags:\\n<tool_call>\\n{\\\"name\\\": <function-name>, "
    "\\\"arguments\\\": <args-json-object>}\\n</tool_call><|im_end|>\\n\" }}\n"
    "{%- else %}\n"
    "    {%- if messages[0]['role'] == 'system' %}\n"
    "        {{- '<|im_start|>system\\n' + messages[0]['content'] + '<|im_end|>\\n' }}\n"
    "    {%- else %}\n"
    "        {{- '<|im_start|>system\\nYou are Qwen, created by Alibaba Cloud. You are a helpful "
    "assistant.<|im_end|>\\n' }}\n"
    "    {%- endif %}\n"
    "{%- endif %}\n"
    "{%- for message in messages %}\n"
    "    {%- if (message.role == \"user\") or (message.role == \"system\" and not loop.first) or "
    "(message.role == \"assistant\" and not message.tool_calls) %}\n"
    "        {{- '<|im_start|>' + message.role + '\\n' + message.content + '<|im_end|>' + '\\n' }}\n"
    "    {%- elif message.role == \"assistant\" %}\n"
    "        {{- '<|im_start|>' + message.role }}\n"
    "        {%- if message.content %}\n"
    "            {{- '\\n' + message.content }}\n"
    "        {%- endif %}\n"
    "        {%- for tool_call in message.tool_calls %}\n"
    "            {%- if tool_call.function is defined %}\n"
    "                {%- set tool_call = tool_call.function %}\n"
    "            {%- endif %}\n"
    "            {{- '\\n<tool_call>\\n{\"name\": \"' }}\n"
    "            {{- tool_call.name }}\n"
    "            {{- '\", \"arguments\": ' }}\n"
    "            {{- tool_call.arguments | tojson }}\n"
    "            {{- '}\\n</tool_call>' }}\n"
    "        {%- endfor %}\n"
    "        {{- '<|im_end|>\\n' }}\n"
    "    {%- elif message.role == \"tool\" %}\n"
    "        {%- if (loop.index0 == 0) or (messages[loop.index0 - 1].role != \"tool\") %}\n"
    "            {{- '<|im_start|>user' }}\n"
    "        {%- endif %}\n"
    "        {{- '\\n<tool_response>\\n' }}\n"
    "        {{- message.content }}\n"
    "        {{- '\\n</tool_response>' }}\n"
    "        {%- if loop.last or (messages[loop.index0 + 1].role != \"tool\") %}\n"
    "            {{- '<|im_end|>\\n' }}\n"
    "        {%- endif %}\n"
    "    {%- endif %}\n"
    "{%- endfor %}\n"
    "{%- if add_generation_prompt %}\n"
    "    {{- '<|im_start|>assistant\\n' }}\n"
    "{%- endif %}\n")


def pre_tokenizer_pattern(meta: Dict[str, Any]) -> str:
    pre = str(meta.get("tokenizer.ggml.pre", "qwen2")).lower()
    if pre not in PRE_TOKENIZERS:
        raise ValueError(f"tokenizer.ggml.pre = {pre!r} is not implemented by this engine "
                         f"(supported: {', '.join(sorted(PRE_TOKENIZERS))}); refusing to load a model "
                         f"whose prompts would be tokenised differently from llama.cpp")
    return PRE_TOKENIZERS[pre]


def message_text(content) -> str:
    """OpenAI content parts → text."""
    if isinstance(content, list):
        return "".join(p.get("text", "") for p in content if isinstance(p, dict))
    return "" if content is None else str(content)


class TemplateError(ValueError):
    pass


class ChatFormatter:
    """``render(messages)`` → the prompt text the model was trained on."""

    def __init__(self, template: Optional[str], bos_token: str = "", eos_token: str = "",
                 default_system: Optional[str] = None):
        self.source = template
        self.bos_token = bos_token
        self.eos_token = eos_token
        self.default_system = default_system
        self._tmpl = None
        if template:
            from jinja2.exceptions import TemplateSyntaxError
            from jinja2.sandbox import ImmutableSandboxedEnvironment

            env = ImmutableSandboxedEnvironment(trim_blocks=True, lstrip_blocks=True)

            def tojson(x, ensure_ascii=False, indent=None, separators=None, sort_keys=False):
                return json.dumps(x, ensure_ascii=ensure_ascii, indent=indent,
                                  separators=separators, sort_keys=sort_keys)

            def raise_exception(msg):
                raise TemplateError(msg)

            env.filters["tojson"] = tojson
            env.globals["raise_exception"] = raise_exception
            env.globals["strftime_now"] = lambda fmt: datetime.datetime.now().strftime(fmt)
            try:
                self._tmpl = env.from_string(template)
            except TemplateSyntaxError as e:
                raise TemplateError(f"tokenizer.chat_template does not parse: {e}") from None

    @classmethod
    def from_gguf(cls, meta: Dict[str, Any], tokens: Optional[Sequence[str]] = None) -> "ChatFormatter":
        def tok(key):
            i = meta.get(key)
            if tokens is None or i is None or not 0 <= int(i) < len(tokens):
                return ""
            return tokens[int(i)]
        from .tokenizer import DEFAULT_SYSTEM

        return cls(meta.get("tokenizer.chat_template"), bos_token=tok("tokenizer.ggml.bos_token_id"),
                   eos_token=tok("tokenizer.ggml.eos_token_id"), default_system=DEFAULT_SYSTEM)

    @property
    def kind(self) -> str:
        return "gguf" if self._tmpl is not None else "chatml-fallback"

    def render(self, messages: Sequence[Dict[str, Any]], add_generation_prompt: bool = True,
               tools: Optional[List[Dict[str, Any]]] = None, **extra) -> str:
        msgs = []
        for m in messages:
            if not isinstance(m, dict):
                raise TemplateError(f"message {m!r} is not an object")
            d = dict(m)
            d["role"] = str(d.get("role", "user"))
            d["content"] = message_text(d.get("content"))
            msgs.append(d)
        if self._tmpl is None:
            from .tokenizer import chatml

            return chatml(msgs, default_system=self.default_system,
                          add_generation_prompt=add_generation_prompt)
        try:
            return self._tmpl.render(messages=msgs, add_generation_prompt=add_generation_prompt,
                                     bos_token=self.bos_token, eos_token=self.eos_token,
                                     tools=tools, **extra)
        except TemplateError:
            raise
        except Exception as e:  # noqa: BLE001 - a template bug is a bad request, not a crash
            raise TemplateError(f"chat template failed: {type(e).__name__}: {e}") from None
