"""Constrained decoding for the llama-server-compatible API: GBNF grammars, JSON mode, JSON schema.

The reference's LLM pod runs upstream ``llama-server`` (reference cluster-config/apps/llm/
deployment.yaml:61,78-84), which constrains generation when a request carries ``grammar`` (GBNF
text), ``json_schema`` or an OpenAI ``response_format`` (``json_object`` / ``json_schema``).  This
module gives the in-tree server the same contract:

* :func:`parse_gbnf` — GBNF (rules ``name ::= ...``, alternatives ``|``, string literals, character
  classes ``[a-z]`` / ``[^...]``, ``.``, groups, ``* + ?`` and ``{m}`` / ``{m,}`` / ``{m,n}``
  repetitions, ``#`` comments) into rules of character elements and rule references; repetitions
  and groups become generated rules, left recursion is rejected.
* :class:`Matcher` — the set-of-stacks recogniser: a *state* is every way the text so far can be
  continued (each stack ends in the next character element to match; the empty stack = the text
  is a complete sentence).  Expansions and character steps are memoised per state, so decoding the
  same kind of output repeatedly is dictionary lookups.
* :class:`TokenTrie` / :class:`GrammarState` — per request: whether a token's bytes (UTF-8 decoded
  incrementally, a code point may straddle tokens) keep the text inside the language, and the mask
  of every allowed token, found by walking the vocabulary's byte trie only along live states.  The
  stop tokens are allowed exactly when the text is complete.
* :func:`json_schema_to_gbnf` — a JSON-schema subset (types, properties/required in declared
  order, items/minItems/maxItems, enum/const, anyOf/oneOf, local ``$ref``, string length bounds) to
  GBNF; a keyword outside the subset raises :class:`GrammarError` naming it (HTTP 400), never a
  silently unconstrained answer.

The scheduler samples as llama.cpp's common sampler does: draw from the request's normal sampler
chain, keep the token when the grammar accepts it, otherwise mask every token the grammar rejects
and draw again (server.py ``Scheduler._sample``).
"""
from __future__ import annotations

import json
import re
import threading
from collections import OrderedDict
from typing import Dict, FrozenSet, Iterable, List, Optional, Sequence, Tuple

CHAR, RULE = 0, 1
MAX_CP = 0x10FFFF


class GrammarError(ValueError):
    """A grammar / schema the server cannot enforce (the request is answered with HTTP 400)."""


# ------------------------------------------------------------------------------------------ GBNF
_ESC = {"n": 10, "t": 9, "r": 13, "\\": 92, '"': 34, "[": 91, "]": 93, "-": 45, "/": 47,
        "'": 39, "0": 0, "b": 8, "f": 12, "^": 94}


class Grammar:
    """``rules[rid]`` = alternatives, each a tuple of elements ``(CHAR, ranges, negated)`` or
    ``(RULE, rid)``; ``root`` the start rule."""

    def __init__(self, rules: List[List[tuple]], names: Dict[str, int], root: int):
        self.rules = rules
        self.names = names
        self.root = root


class _Parser:
    def __init__(self, src: str):
        self.s = src
        self.i = 0
        self.names: Dict[str, int] = {}
        self.rules: List[Optional[List[tuple]]] = []
        self.refs: Dict[str, int] = {}           # name -> offset of a first reference

    # ---- lexing
    def err(self, msg: str) -> GrammarError:
        line = self.s.count("\n", 0, self.i) + 1
        return GrammarError(f"grammar line {line}: {msg}")

    def peek(self) -> str:
        return self.s[self.i] if self.i < len(self.s) else ""

    def space(self, newlines: bool) -> None:
        while self.i < len(self.s):
            c = self.s[self.i]
            if c == "#":
                while self.i < len(self.s) and self.s[self.i] not in "\r\n":
                    self.i += 1
            elif c in " \t" or (newlines and c in "\r\n"):
                self.i += 1
            else:
                return

    def name(self) -> str:
        m = re.compile(r"[A-Za-z0-9_-]+").match(self.s, self.i)
        if not m:
            raise self.err(f"expected a rule name at {self.s[self.i:self.i + 12]!r}")
        self.i = m.end()
        return m.group(0)

    def char(self) -> int:
        """One (possibly escaped) character of a literal or class."""
        if self.i >= len(self.s):
            raise self.err("unexpected end of grammar")
        c = self.s[self.i]
        if c != "\\":
            self.i += 1
            return ord(c)
        if self.i + 1 >= len(self.s):
            raise self.err("dangling escape")
        e = self.s[self.i + 1]
        if e in "xuU":
            n = {"x": 2, "u": 4, "U": 8}[e]
            h = self.s[self.i + 2:self.i + 2 + n]
            if len(h) != n or not all(x in "0123456789abcdefABCDEF" for x in h):
                raise self.err(f"bad \\{e} escape")
            self.i += 2 + n
            return int(h, 16)
        if e not in _ESC:
            raise self.err(f"unknown escape \\{e}")
        self.i += 2
        return _ESC[e]

    # ---- rules
    def rid(self, name: str) -> int:
        r = self.names.get(name)
        if r is None:
            r = self.names[name] = len(self.rules)
            self.rules.append(None)
        return r

    def fresh(self, base: str, alts: List[tuple]) -> int:
        k = 1
        while f"{base}-{k}" in self.names:
            k += 1
        r = self.rid(f"{base}-{k}")
        self.rules[r] = alts
        return r

    def parse(self) -> Grammar:
        self.space(True)
        while self.i < len(self.s):
            name = self.name()
            self.space(False)
            if not self.s.startswith("::=", self.i):
                raise self.err(f"expected '::=' after {name!r}")
            self.i += 3
            self.space(True)
            r = self.rid(name)
            if self.rules[r] is not None:
                raise self.err(f"rule {name!r} defined twice")
            self.rules[r] = self.alternates(name, nested=False)
            self.space(True)
        for n, r in self.names.items():
            if self.rules[r] is None:
                raise GrammarError(f"grammar: rule {n!r} is used but never defined")
        if "root" not in self.names:
            raise GrammarError("grammar: no 'root' rule")
        g = Grammar([list(a) for a in self.rules], dict(self.names), self.names["root"])
        _check_left_recursion(g)
        return g

    def alternates(self, name: str, nested: bool) -> List[tuple]:
        alts = [tuple(self.sequence(name, nested))]
        while self.peek() == "|":
            self.i += 1
            self.space(True)
            alts.append(tuple(self.sequence(name, nested)))
        return alts

    def sequence(self, name: str, nested: bool) -> List[tuple]:
        out: List[tuple] = []
        last = len(out)
        while self.i < len(self.s):
            c = self.peek()
            if c == '"':
                self.i += 1
                last = len(out)
                while self.peek() != '"':
                    if not self.peek():
                        raise self.err("unterminated string literal")
                    cp = self.char()
                    out.append((CHAR, ((cp, cp),), False))
                self.i += 1
            elif c == "[":
                self.i += 1
                neg = self.peek() == "^"
                if neg:
                    self.i += 1
                ranges = []
                while self.peek() != "]":
                    if not self.peek():
                        raise self.err("unterminated character class")
                    lo = self.char()
                    hi = lo
                    if self.peek() == "-" and self.s[self.i + 1:self.i + 2] not in ("]", ""):
                        self.i += 1
                        hi = self.char()
                    if hi < lo:
                        raise self.err("empty character range")
                    ranges.append((lo, hi))
                self.i += 1
                last = len(out)
                out.append((CHAR, tuple(ranges), neg))
            elif c == ".":
                self.i += 1
                last = len(out)
                out.append((CHAR, ((0, MAX_CP),), False))
            elif c == "(":
                self.i += 1
                self.space(True)
                alts = self.alternates(name, nested=True)
                if self.peek() != ")":
                    raise self.err("expected ')'")
                self.i += 1
                last = len(out)
                out.append((RULE, self.fresh(name, alts)))
            elif re.match(r"[A-Za-z0-9_-]", c):
                ref = self.name()
                save = self.i
                self.space(False)
                if self.s.startswith("::=", self.i):
                    raise self.err(f"missing newline before rule {ref!r}")
                self.i = save
                last = len(out)
                out.append((RULE, self.rid(ref)))
            elif c in "*+?{":
                if last == len(out):
                    raise self.err(f"'{c}' without a preceding element")
                lo, hi = self.repetition()
                seq = tuple(out[last:])
                del out[last:]
                out.extend(self.repeat(name, seq, lo, hi))
                last = len(out)          # a repetition is not itself repeatable without a group
            else:
                break
            self.space(nested)
        return out

    def repetition(self) -> Tuple[int, Optional[int]]:
        c = self.s[self.i]
        self.i += 1
        if c == "*":
            return 0, None
        if c == "+":
            return 1, None
        if c == "?":
            return 0, 1
        m = re.compile(r"\s*(\d+)\s*(?:(,)\s*(\d*)\s*)?\}").match(self.s, self.i)
        if not m:
            raise self.err("bad {m,n} repetition")
        self.i = m.end()
        lo = int(m.group(1))
        hi = lo if m.group(2) is None else (int(m.group(3)) if m.group(3) else None)
        if hi is not None and hi < lo:
            raise self.err("repetition {m,n} with n < m")
        return lo, hi

    def repeat(self, name: str, seq: tuple, lo: int, hi: Optional[int]) -> List[tuple]:
        out = list(seq) * lo
        if hi is None:               # R ::= seq R | (empty)   (right recursion: no stack growth)
            r = self.fresh(name, [])
            self.rules[r] = [seq + ((RULE, r),), ()]
            out.append((RULE, r))
        elif hi > lo:                # nested optionals: (seq (seq (...)?)?)?
            tail: Optional[int] = None
            for _ in range(hi - lo):
                body = seq + (((RULE, tail),) if tail is not None else ())
                tail = self.fresh(name, [body, ()])
            out.append((RULE, tail))
        return out


def _check_left_recursion(g: Grammar) -> None:
    """A rule that can reach itself without consuming a character would expand forever."""
    n = len(g.rules)
    nullable = [False] * n
    changed = True
    while changed:
        changed = False
        for r, alts in enumerate(g.rules):
            if nullable[r]:
                continue
            if any(all(e[0] == RULE and nullable[e[1]] for e in alt) for alt in alts):
                nullable[r] = changed = True
    left: List[set] = [set() for _ in range(n)]
    for r, alts in enumerate(g.rules):
        for alt in alts:
            for e in alt:
                if e[0] == CHAR:
                    break
                left[r].add(e[1])
                if not nullable[e[1]]:
                    break
    names = {v: k for k, v in g.names.items()}
    state = [0] * n                  # 0 new, 1 on the DFS path, 2 done

    def visit(r):
        stack = [(r, iter(left[r]))]
        state[r] = 1
        while stack:
            node, it = stack[-1]
            nxt = next(it, None)
            if nxt is None:
                state[node] = 2
                stack.pop()
            elif state[nxt] == 1:
                raise GrammarError(f"grammar: left recursion through rule {names.get(nxt, nxt)!r}")
            elif state[nxt] == 0:
                state[nxt] = 1
                stack.append((nxt, iter(left[nxt])))

    for r in range(n):
        if state[r] == 0:
            visit(r)


def parse_gbnf(src: str) -> Grammar:
    if not isinstance(src, str) or not src.strip():
        raise GrammarError("grammar must be a non-empty GBNF string")
    return _Parser(src).parse()


# ------------------------------------------------------------------------------------------ matcher
Stack = Tuple[Tuple[int, int, int], ...]
Stacks = FrozenSet[Stack]
State = Tuple[Stacks, bytes]          # (stacks, pending bytes of an incomplete UTF-8 sequence)


def _utf8_len(lead: int) -> int:
    return 2 if lead < 0xE0 else 3 if lead < 0xF0 else 4


class Matcher:
    """Set-of-stacks recogniser of one grammar with memoised expansions and steps."""

    MAX_CACHE = 1 << 18

    def __init__(self, g: Grammar):
        self.g = g
        self._exp: Dict[Stack, Stacks] = {}
        self._step: Dict[tuple, Stacks] = {}
        self._byte: Dict[tuple, Optional[State]] = {}
        self._allowed: "OrderedDict[tuple, List[int]]" = OrderedDict()
        self._lock = threading.Lock()
        start: set = set()
        for a, alt in enumerate(g.rules[g.root]):
            start |= self._expand(((g.root, a, 0),) if alt else ())
        self.start: State = (frozenset(start), b"")

    def _expand(self, stack: Stack) -> Stacks:
        hit = self._exp.get(stack)
        if hit is not None:
            return hit
        rules = self.g.rules
        out = set()
        work = [stack]
        while work:
            s = work.pop()
            if not s:
                out.add(())
                continue
            r, a, i = s[-1]
            alt = rules[r][a]
            el = alt[i]
            if el[0] == CHAR:
                out.add(s)
                continue
            rest = s[:-1] + (((r, a, i + 1),) if i + 1 < len(alt) else ())
            for a2, alt2 in enumerate(rules[el[1]]):
                work.append(rest + ((el[1], a2, 0),) if alt2 else rest)
        fs = frozenset(out)
        if len(self._exp) < self.MAX_CACHE:
            self._exp[stack] = fs
        return fs

    def step(self, stacks: Stacks, cp: int) -> Stacks:
        """Stacks after one code point (empty: the text left the language)."""
        key = (stacks, cp)
        hit = self._step.get(key)
        if hit is not None:
            return hit
        rules = self.g.rules
        out: set = set()
        for s in stacks:
            if not s:
                continue
            r, a, i = s[-1]
            alt = rules[r][a]
            _, ranges, neg = alt[i]
            ok = False
            for lo, hi in ranges:
                if lo <= cp <= hi:
                    ok = True
                    break
            if ok != neg:
                out |= self._expand(s[:-1] + (((r, a, i + 1),) if i + 1 < len(alt) else ()))
        fs = frozenset(out)
        if len(self._step) < self.MAX_CACHE:
            self._step[key] = fs
        return fs

    def byte(self, state: State, b: int) -> Optional[State]:
        """State after one byte of UTF-8 text; None when no continuation exists."""
        key = (state, b)
        if key in self._byte:
            return self._byte[key]
        stacks, pend = state
        nxt: Optional[State]
        if pend:
            if not 0x80 <= b < 0xC0:
                nxt = None
            else:
                pend = pend + bytes((b,))
                if len(pend) < _utf8_len(pend[0]):
                    nxt = (stacks, pend) if self._possible(stacks, pend) else None
                else:
                    try:
                        cp = ord(pend.decode("utf-8"))
                    except UnicodeDecodeError:
                        cp = -1
                    st = self.step(stacks, cp) if cp >= 0 else frozenset()
                    nxt = (st, b"") if st else None
        elif b < 0x80:
            st = self.step(stacks, b)
            nxt = (st, b"") if st else None
        elif 0xC2 <= b <= 0xF4:
            nxt = (stacks, bytes((b,))) if self._possible(stacks, bytes((b,))) else None
        else:
            nxt = None
        if len(self._byte) < self.MAX_CACHE:
            self._byte[key] = nxt
        return nxt

    def _possible(self, stacks: Stacks, pend: bytes) -> bool:
        """Can some code point that starts with the bytes ``pend`` be matched next?"""
        n = _utf8_len(pend[0])
        lo = pend[0] & (0x7F >> n)
        for c in pend[1:]:
            lo = (lo << 6) | (c & 0x3F)
        lo <<= 6 * (n - len(pend))
        hi = lo | ((1 << (6 * (n - len(pend)))) - 1)
        lo = max(lo, (0x80, 0x800, 0x10000)[n - 2])      # shortest form only (no overlongs)
        hi = min(hi, MAX_CP)
        if lo > hi:
            return False
        rules = self.g.rules
        for s in stacks:
            if not s:
                continue
            r, a, i = s[-1]
            _, ranges, neg = rules[r][a][i]
            if not neg:
                if any(x <= hi and y >= lo for x, y in ranges):
                    return True
                continue
            # negated class: possible unless its ranges cover all of [lo, hi]
            cur = lo
            for x, y in sorted(ranges):
                if x > cur:
                    break
                cur = max(cur, y + 1)
                if cur > hi:
                    break
            if cur <= hi:
                return True
        return False

    def feed(self, state: State, data: bytes) -> Optional[State]:
        for b in data:
            state = self.byte(state, b)
            if state is None:
                return None
        return state

    @staticmethod
    def complete(state: State) -> bool:
        return not state[1] and () in state[0]

    @staticmethod
    def only_complete(state: State) -> bool:
        return not state[1] and state[0] == frozenset({()})


class TokenTrie:
    """Byte trie of a vocabulary (tokens with no bytes — control tokens — are left out)."""

    def __init__(self, token_bytes: Sequence[bytes]):
        self.children: List[Dict[int, int]] = [{}]
        self.ends: List[List[int]] = [[]]
        for tid, bs in enumerate(token_bytes):
            if not bs:
                continue
            n = 0
            for b in bs:
                ch = self.children[n]
                nxt = ch.get(b)
                if nxt is None:
                    nxt = ch[b] = len(self.children)
                    self.children.append({})
                    self.ends.append([])
                n = nxt
            self.ends[n].append(tid)

    def allowed(self, m: Matcher, state: State) -> List[int]:
        out: List[int] = []
        work = [(0, state)]
        children, ends = self.children, self.ends
        while work:
            node, st = work.pop()
            for b, child in children[node].items():
                st2 = m.byte(st, b)
                if st2 is None:
                    continue
                if ends[child]:
                    out.extend(ends[child])
                if children[child]:
                    work.append((child, st2))
        return out


_TRIES: "OrderedDict[int, TokenTrie]" = OrderedDict()
_GRAMMARS: "OrderedDict[str, Matcher]" = OrderedDict()
_cache_lock = threading.Lock()


def trie_for(tok) -> TokenTrie:
    """The vocabulary trie of a tokenizer, built once (``tok.token_bytes()``)."""
    key = id(tok)
    with _cache_lock:
        t = _TRIES.get(key)
        if t is None:
            t = _TRIES[key] = TokenTrie(tok.token_bytes())
            while len(_TRIES) > 4:
                _TRIES.popitem(last=False)
        return t


def matcher_for(src: str) -> Matcher:
    """A compiled grammar, shared (with its memo tables) by every request sending the same text."""
    with _cache_lock:
        m = _GRAMMARS.get(src)
        if m is not None:
            _GRAMMARS.move_to_end(src)
            return m
    m = Matcher(parse_gbnf(src))
    with _cache_lock:
        _GRAMMARS[src] = m
        while len(_GRAMMARS) > 32:
            _GRAMMARS.popitem(last=False)
    return m


class GrammarState:
    """One request's position in its grammar, over a tokenizer's vocabulary."""

    MASK_CACHE = 128

    def __init__(self, matcher: Matcher, tok, stop_ids: Iterable[int]):
        self.m = matcher
        self.tok = tok
        self.tb = tok.token_bytes()
        self.stop_ids = sorted(set(int(s) for s in stop_ids))
        self.state: State = matcher.start
        self._masks: "OrderedDict[tuple, object]" = OrderedDict()

    def accepts(self, tid: int) -> bool:
        if tid in self.stop_ids:
            return self.m.complete(self.state)
        bs = self.tb[tid] if 0 <= tid < len(self.tb) else b""
        return bool(bs) and self.m.feed(self.state, bs) is not None

    def advance(self, tid: int) -> None:
        if tid in self.stop_ids:
            return
        nxt = self.m.feed(self.state, self.tb[tid])
        if nxt is None:
            raise GrammarError(f"token {tid} is not allowed by the grammar here")
        self.state = nxt

    @property
    def finished(self) -> bool:
        """Only the end of the text is left: the next token must be a stop token."""
        return self.m.only_complete(self.state)

    def allowed_ids(self) -> List[int]:
        """Every token id allowed next.  The walk is memoised on the grammar (shared by every
        request using it), keyed by state and vocabulary: a permissive state (inside a JSON
        string, ~all of a 152k vocabulary) costs one walk of the whole trie (~0.7 s) the first
        time, then nothing."""
        trie = trie_for(self.tok)
        key = (self.state, id(trie))
        with self.m._lock:
            ids = self.m._allowed.get(key)
            if ids is not None:
                self.m._allowed.move_to_end(key)
        if ids is None:
            ids = trie.allowed(self.m, self.state)
            with self.m._lock:
                self.m._allowed[key] = ids
                while len(self.m._allowed) > 64:
                    self.m._allowed.popitem(last=False)
        if self.m.complete(self.state):
            ids = ids + self.stop_ids
        return ids

    def mask(self, vocab: int, device):
        """bool [vocab] of the tokens allowed next (memoised per grammar state)."""
        import torch

        key = (self.state, str(device), vocab)
        hit = self._masks.get(key)
        if hit is not None:
            self._masks.move_to_end(key)
            return hit
        m = torch.zeros(vocab, dtype=torch.bool)
        ids = [i for i in self.allowed_ids() if i < vocab]
        if ids:
            m[torch.tensor(ids, dtype=torch.long)] = True
        m = m.to(device)
        self._masks[key] = m
        while len(self._masks) > self.MASK_CACHE:
            self._masks.popitem(last=False)
        return m


# --------------------------------------------------------------------------------------- JSON
_JSON_PRIMITIVES = r'''
ws ::= | " " | "\n" [ \t]{0,8}
string ::= "\"" char* "\"" ws
char ::= [^"\\\x00-\x1F\x7F] | "\\" (["\\/bfnrt] | "u" [0-9a-fA-F]{4})
number ::= "-"? ("0" | [1-9] [0-9]{0,15}) ("." [0-9]{1,16})? ([eE] [-+]? [0-9]{1,4})? ws
integer ::= "-"? ("0" | [1-9] [0-9]{0,15}) ws
boolean ::= ("true" | "false") ws
null ::= "null" ws
value ::= object | array | string | number | boolean | null
object ::= "{" ws ( string ":" ws value ( "," ws string ":" ws value )* )? "}" ws
array ::= "[" ws ( value ( "," ws value )* )? "]" ws
'''

JSON_OBJECT_GBNF = "root ::= object\n" + _JSON_PRIMITIVES

_ANNOTATIONS = {"title", "description", "default", "examples", "$schema", "$id", "$comment",
                "readOnly", "writeOnly", "deprecated", "$defs", "definitions"}


def _lit(s: str) -> str:
    """A GBNF string literal matching ``s`` exactly."""
    out = []
    for ch in s:
        o = ord(ch)
        if ch in '"\\':
            out.append("\\" + ch)
        elif o < 0x20 or o == 0x7F:
            out.append(f"\\x{o:02X}")
        else:
            out.append(ch)
    return '"' + "".join(out) + '"'


class _SchemaConv:
    def __init__(self, root: dict):
        self.root = root
        self.rules: "OrderedDict[str, str]" = OrderedDict()
        self.refs: Dict[str, str] = {}

    def name(self, hint: str) -> str:
        base = re.sub(r"[^A-Za-z0-9-]+", "-", hint).strip("-") or "r"
        n, k = base, 1
        while n in self.rules or n in ("ws", "string", "char", "number", "integer", "boolean",
                                        "null", "value", "object", "array", "root"):
            k += 1
            n = f"{base}-{k}"
        self.rules[n] = ""
        return n

    def rule(self, hint: str, body: str) -> str:
        n = self.name(hint)
        self.rules[n] = body
        return n

    def visit(self, s, hint: str, path: str) -> str:
        """GBNF expression (one element) for schema ``s``."""
        if s is True or s == {}:
            return "value"
        if s is False or not isinstance(s, dict):
            raise GrammarError(f"{path}: unsupported schema {s!r}")
        if "$ref" in s:
            return self.ref(s["$ref"], path)
        for k in s:
            if k not in _ANNOTATIONS and k not in (
                    "type", "properties", "required", "additionalProperties", "items", "minItems",
                    "maxItems", "enum", "const", "anyOf", "oneOf", "allOf", "minLength",
                    "maxLength", "nullable", "strict"):
                raise GrammarError(f"{path}: unsupported JSON-schema keyword {k!r}")
        if "const" in s:
            return self.rule(hint, _lit(json.dumps(s["const"], ensure_ascii=False)) + " ws")
        if "enum" in s:
            if not isinstance(s["enum"], list) or not s["enum"]:
                raise GrammarError(f"{path}.enum must be a non-empty list")
            alts = " | ".join(_lit(json.dumps(v, ensure_ascii=False)) for v in s["enum"])
            return self.rule(hint, f"({alts}) ws")
        for key in ("anyOf", "oneOf"):
            if key in s:
                subs = s[key]
                if not isinstance(subs, list) or not subs:
                    raise GrammarError(f"{path}.{key} must be a non-empty list")
                alts = [self.visit(x, f"{hint}-{i}", f"{path}.{key}[{i}]") for i, x in enumerate(subs)]
                return self.rule(hint, " | ".join(alts))
        if "allOf" in s:
            subs = s["allOf"]
            if not isinstance(subs, list) or len(subs) != 1:
                raise GrammarError(f"{path}.allOf: only a single subschema is supported")
            return self.visit(subs[0], hint, f"{path}.allOf[0]")
        t = s.get("type")
        if isinstance(t, list):
            alts = [self.visit(dict(s, type=x), f"{hint}-{x}", path) for x in t]
            return self.rule(hint, " | ".join(alts))
        if s.get("nullable") and t is not None:
            inner = self.visit({k: v for k, v in s.items() if k != "nullable"}, hint, path)
            return self.rule(hint, f"{inner} | null")
        if t is None:
            if "properties" in s:
                t = "object"
            elif "items" in s:
                t = "array"
            else:
                return "value"
        if t == "string":
            lo, hi = s.get("minLength"), s.get("maxLength")
            if lo is None and hi is None:
                return "string"
            lo = int(lo or 0)
            rep = f"{{{lo},{int(hi)}}}" if hi is not None else f"{{{lo},}}"
            return self.rule(hint, f'"\\"" char{rep} "\\"" ws')
        if t in ("number", "integer", "boolean", "null"):
            return t
        if t == "array":
            item = self.visit(s.get("items", True), f"{hint}-item", f"{path}.items")
            lo = int(s.get("minItems", 0))
            hi = s.get("maxItems")
            if hi is not None and int(hi) < lo:
                raise GrammarError(f"{path}: maxItems < minItems")
            if hi is not None and int(hi) == 0:
                return self.rule(hint, '"[" ws "]" ws')
            more_lo = max(lo - 1, 0)
            rep = f"{{{more_lo},{int(hi) - 1}}}" if hi is not None else (
                f"{{{more_lo},}}" if more_lo else "*")
            body = f'{item} ("," ws {item}){rep}'
            body = f'"[" ws {body} "]" ws' if lo > 0 else f'"[" ws ({body})? "]" ws'
            return self.rule(hint, body)
        if t == "object":
            props = s.get("properties")
            if not props:
                extra = s.get("additionalProperties", True)
                val = self.visit(extra if extra is not False else True, f"{hint}-value",
                                 f"{path}.additionalProperties")
                if extra is False:
                    return self.rule(hint, '"{" ws "}" ws')
                return self.rule(hint, f'"{{" ws ( string ":" ws {val} ( "," ws string ":" ws '
                                       f'{val} )* )? "}}" ws')
            if not isinstance(props, dict):
                raise GrammarError(f"{path}.properties must be an object")
            req = s.get("required", [])
            if not isinstance(req, list) or any(r not in props for r in req):
                raise GrammarError(f"{path}.required names a property not in properties")
            keys = list(props)
            kv = [self.rule(f"{hint}-{k}-kv",
                            f'{_lit(json.dumps(k, ensure_ascii=False))} ws ":" ws '
                            f'{self.visit(props[k], f"{hint}-{k}", f"{path}.properties.{k}")}')
                  for k in keys]
            # S(i, first): the properties from i on, in declared order, required ones mandatory
            names: Dict[tuple, str] = {}
            for i in range(len(keys), -1, -1):
                for first in (True, False):
                    names[(i, first)] = self.name(f"{hint}-s{i}{'f' if first else ''}")
            for i in range(len(keys), -1, -1):
                for first in (True, False):
                    n = names[(i, first)]
                    if i == len(keys):
                        self.rules[n] = '""'         # (a bare "::=" would run into the next line)
                        continue
                    sep = "" if first else '"," ws '
                    take = f"{sep}{kv[i]} {names[(i + 1, False)]}"
                    self.rules[n] = take if keys[i] in req else f"{take} | {names[(i + 1, first)]}"
            return self.rule(hint, f'"{{" ws {names[(0, True)]} "}}" ws')
        raise GrammarError(f"{path}: unsupported type {t!r}")

    def ref(self, ref: str, path: str) -> str:
        if ref in self.refs:
            return self.refs[ref]
        m = re.fullmatch(r"#/(\$defs|definitions)/([^/]+)", str(ref))
        if not m or m.group(2) not in (self.root.get(m.group(1)) or {}):
            raise GrammarError(f"{path}: unsupported or unresolvable $ref {ref!r}")
        n = self.name(f"def-{m.group(2)}")
        self.refs[ref] = n
        self.rules[n] = self.visit(self.root[m.group(1)][m.group(2)], f"{n}-body",
                                   f"{path}->{ref}")
        return n


def json_schema_to_gbnf(schema) -> str:
    """GBNF text for a JSON-schema subset (see the module docstring); GrammarError otherwise."""
    if isinstance(schema, str):
        try:
            schema = json.loads(schema)
        except ValueError as e:
            raise GrammarError(f"json_schema is not valid JSON: {e}") from None
    conv = _SchemaConv(schema if isinstance(schema, dict) else {})
    top = conv.visit(schema, "root-value", "json_schema")
    lines = [f"root ::= {top}"]
    for n, body in conv.rules.items():
        lines.append(f"{n} ::= {body}")
    return "\n".join(lines) + "\n" + _JSON_PRIMITIVES


def grammar_from_request(body: dict) -> Optional[str]:
    """The GBNF a llama-server / OpenAI request asks for, or None.  Sources: ``grammar`` (GBNF
    text), ``json_schema`` (llama-server), ``response_format`` {"type": "json_object"
    [, "schema"]} / {"type": "json_schema", "json_schema": {"schema": ...}} / {"type": "text"}.
    More than one source, or a malformed one, raises GrammarError (HTTP 400)."""
    srcs = []
    g = body.get("grammar")
    if g not in (None, ""):
        if not isinstance(g, str):
            raise GrammarError("grammar must be a GBNF string")
        srcs.append(("grammar", g))
    js = body.get("json_schema")
    if js not in (None, {}):
        srcs.append(("json_schema", json_schema_to_gbnf(js)))
    rf = body.get("response_format")
    if rf not in (None, {}):
        if not isinstance(rf, dict):
            raise GrammarError("response_format must be an object")
        kind = rf.get("type")
        if kind == "json_object":
            srcs.append(("response_format", json_schema_to_gbnf(rf["schema"]) if rf.get("schema")
                         else JSON_OBJECT_GBNF))
        elif kind == "json_schema":
            inner = rf.get("json_schema")
            schema = inner.get("schema") if isinstance(inner, dict) else None
            if schema is None:
                schema = rf.get("schema")
            if schema is None:
                raise GrammarError("response_format.json_schema.schema is missing")
            srcs.append(("response_format", json_schema_to_gbnf(schema)))
        elif kind != "text":
            raise GrammarError(f"response_format.type {kind!r} is not supported "
                               "(text, json_object, json_schema)")
    if len(srcs) > 1:
        raise GrammarError("only one of grammar / json_schema / response_format may be given "
                           f"(got {', '.join(k for k, _ in srcs)})")
    if not srcs:
        return None
    matcher_for(srcs[0][1])          # parse now: a bad grammar is the request's 400
    return srcs[0][1]
