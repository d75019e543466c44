"""A minimal Go text/template evaluator for the offline tests of RKE2's containerd templates.

RKE2 renders ``config-v3.toml.tmpl`` with Go's ``text/template`` (the k3s agent templates) and
our Ansible role writes a Jinja template that emits that Go template (see
``rke2-installation/roles/amd-host-prep/templates/config-v3.toml.tmpl.j2``).  No Go toolchain is
available here, so this module implements the subset those templates use: ``{{ template "base" . }}``,
field chains (``.A.B``, ``$.A``, ``$v.A``, ``.``), ``printf "%q"``, ``or``, ``eq``, ``deschemify``,
pipelines, ``if``/``else``/``with``/``range $k, $v :=``/``end``, comments and ``{{-``/``-}}`` trim
markers.  Anything else raises, so a template edit that needs more fails loudly instead of
rendering wrong.
"""
from __future__ import annotations

import json
import re
import shlex
from typing import Any, Dict, List, Optional, Tuple

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


def _tokens(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        if out and out[-1][0] == "rtrim":
            out.pop()
            text = text.lstrip()
        out.append(("text", text))
        body = m.group(2)
        if not (body.startswith("/*") and body.endswith("*/")):
            out.append(("action", body))
        if m.group(3):
            out.append(("rtrim", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "rtrim":
        out.pop()
        text = text.lstrip()
    out.append(("text", text))
    return out


class _Node:
    def __init__(self, kind: str, arg: str = ""):
        self.kind, self.arg = kind, arg
        self.body: List[Any] = []
        self.other: List[Any] = []


def _parse(tokens: List[Tuple[str, str]]) -> List[Any]:
    root: List[Any] = []
    stack: List[Tuple[_Node, bool]] = []

    def sink() -> List[Any]:
        if not stack:
            return root
        node, in_else = stack[-1]
        return node.other if in_else else node.body

    for kind, val in tokens:
        if kind == "text":
            if val:
                sink().append(val)
            continue
        word = val.split(None, 1)[0] if val else ""
        rest = val[len(word):].strip()
        if word in ("if", "with", "range"):
            node = _Node(word, rest)
            sink().append(node)
            stack.append((node, False))
        elif word == "else":
            node, _ = stack.pop()
            stack.append((node, True))
        elif word == "end":
            stack.pop()
        else:
            sink().append(_Node("expr", val))
    if stack:
        raise ValueError("unterminated block")
    return root


def _split_words(expr: str) -> List[str]:
    lex = shlex.shlex(expr, posix=False)
    lex.whitespace_split = True
    lex.commenters = ""
    return list(lex)


class Renderer:
    def __init__(self, templates: Dict[str, str]):
        self.templates = {k: _parse(_tokens(v)) for k, v in templates.items()}

    def render(self, name: str, ctx: Any) -> str:
        return self._run(self.templates[name], ctx, ctx, {})

    # ------------------------------------------------------------ evaluation
    def _field(self, obj: Any, chain: List[str]) -> Any:
        for f in chain:
            if f == "":
                continue
            obj = obj.get(f) if isinstance(obj, dict) else getattr(obj, f)
        return obj

    def _atom(self, w: str, dot: Any, root: Any, vars_: Dict[str, Any]) -> Any:
        if w.startswith('"'):
            return json.loads(w)
        if w in ("true", "false"):
            return w == "true"
        if w == ".":
            return dot
        if w.startswith("."):
            return self._field(dot, w[1:].split("."))
        if w.startswith("$"):
            head, *chain = w.split(".")
            base = root if head == "$" else vars_[head]
            return self._field(base, chain)
        raise ValueError(f"unsupported operand {w!r}")

    def _call(self, words: List[str], dot, root, vars_, piped=None) -> Any:
        fn = words[0]
        args = [self._atom(w, dot, root, vars_) for w in words[1:]]
        if piped is not None:
            args.append(piped[0])
        if fn == "printf":
            if args[0] != "%q":
                raise ValueError("only printf %q is supported")
            return json.dumps(str(args[1]))
        if fn == "or":
            for a in args:
                if a:
                    return a
            return args[-1]
        if fn == "eq":
            return args[0] == args[1]
        if fn == "not":
            return not args[0]
        if fn == "deschemify":
            return re.sub(r"^[a-z]+://", "", str(args[0]))
        if not words[1:] and piped is None:
            return self._atom(fn, dot, root, vars_)
        raise ValueError(f"unsupported function {fn!r}")

    def _eval(self, expr: str, dot, root, vars_) -> Any:
        stages = [s.strip() for s in expr.split("|")]
        val = None
        for i, st in enumerate(stages):
            words = _split_words(st)
            if i == 0:
                val = (self._call(words, dot, root, vars_) if len(words) > 1
                       else self._atom(words[0], dot, root, vars_))
            else:
                val = self._call(words, dot, root, vars_, piped=(val,))
        return val

    @staticmethod
    def _fmt(v: Any) -> str:
        if isinstance(v, bool):
            return "true" if v else "false"
        return "" if v is None else str(v)

    def _run(self, nodes: List[Any], dot, root, vars_) -> str:
        out: List[str] = []
        for n in nodes:
            if isinstance(n, str):
                out.append(n)
            elif n.kind == "expr":
                m = re.fullmatch(r'template\s+"([^"]+)"\s+(\S+)', n.arg)
                if m:
                    out.append(self._run(self.templates[m.group(1)], self._atom(m.group(2), dot, root,
                                                                                  vars_), root, vars_))
                else:
                    out.append(self._fmt(self._eval(n.arg, dot, root, vars_)))
            elif n.kind == "if":
                cond = self._eval(n.arg, dot, root, vars_)
                out.append(self._run(n.body if cond else n.other, dot, root, vars_))
            elif n.kind == "with":
                v = self._eval(n.arg, dot, root, vars_)
                out.append(self._run(n.body, v, root, vars_) if v else self._run(n.other, dot, root, vars_))
            elif n.kind == "range":
                m = re.fullmatch(r"(\$\w+)\s*,\s*(\$\w+)\s*:=\s*(.+)", n.arg)
                if not m:
                    raise ValueError(f"unsupported range {n.arg!r}")
                coll = self._eval(m.group(3), dot, root, vars_) or {}
                for k in sorted(coll):
                    v2 = dict(vars_, **{m.group(1): k, m.group(2): coll[k]})
                    out.append(self._run(n.body, coll[k], root, v2))
            else:  # pragma: no cover
                raise ValueError(n.kind)
        return "".join(out)


def render(templates: Dict[str, str], name: str, ctx: Any) -> str:
    return Renderer(templates).render(name, ctx)


def rke2_context(systemd_cgroup: bool = True, default_runtime: Optional[str] = None,
                 extra_runtimes: Optional[Dict[str, Dict[str, str]]] = None) -> Dict[str, Any]:
    """Stub of the fields RKE2 v1.32 passes to the containerd template on a RHEL8 server node."""
    return {
        "Program": "rke2",
        "SystemdCgroup": systemd_cgroup,
        "EnableUnprivileged": True,
        "NonrootDevices": False,
        "DisableCgroup": False,
        "IsRunningInUserNS": False,
        "ExtraRuntimes": extra_runtimes or {},
        "PrivateRegistryConfig": None,
        "NodeConfig": {
            "SELinux": False,
            "DefaultRuntime": default_runtime or "",
            "NoFlannel": True,
            "Containerd": {
                "Root": "/var/lib/rancher/rke2/agent/containerd",
                "State": "/run/k3s/containerd",
                "Address": "unix:///run/k3s/containerd/containerd.sock",
                "Opt": "/var/lib/rancher/rke2/agent/containerd",
                "Registry": "/var/lib/rancher/rke2/agent/etc/containerd/certs.d",
            },
            "AgentConfig": {
                "Snapshotter": "overlayfs",
                "PauseImage": "index.docker.io/rancher/mirrored-pause:3.6",
                "CNIBinDir": "/var/lib/rancher/rke2/data/current/bin",
                "CNIConfDir": "/var/lib/rancher/rke2/agent/etc/cni/net.d",
            },
        },
    }
