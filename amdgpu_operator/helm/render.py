"""Minimal Helm chart renderer for the subset of Go templates the chart uses.

There is no ``helm`` binary in the build environment, so the
chart (``deploy/helm/amd-gpu-operator``) is rendered here for tests, for the
``amdgpu-operator install`` dry-run and for the simulated cluster.  Supported:

* actions ``{{ ... }}`` with ``{{-`` / ``-}}`` whitespace trimming;
* ``if`` / ``else if`` / ``else`` / ``end``, ``with`` / ``end``, ``range`` over lists,
  ``define`` / ``include``;
* values ``.Values.a.b``, ``.Release.Name|Namespace|Service``, ``.Chart.Name|Version|AppVersion``,
  ``.`` (scope), string / number / bool literals;
* functions ``toYaml``, ``nindent``, ``indent``, ``quote``, ``default``, ``not``,
  ``and``, ``or``, ``eq``, ``ne``, ``printf`` (%s %d), ``trunc``, ``trimSuffix``,
  ``include``; pipelines ``a | f b``.

The same values file drives the real ``helm install`` of the reference's
command line (/root/reference/README.md:101-110).
"""

from __future__ import annotations

import os
import re
import shlex

import yaml

# libyaml's safe loader when PyYAML was built with it (the CRD parses ~10x faster), else the pure-Python one
_Loader = getattr(yaml, "CSafeLoader", yaml.SafeLoader)

from ..api.clusterpolicy import deep_merge, parse_set_flags

CHART_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                         "deploy", "helm", "amd-gpu-operator")

_ACTION = re.compile(r"\{\{(-?)\s*(.*?)\s*(-?)\}\}", re.S)


class TemplateError(Exception):
    pass


def _tokenize(src: str):
    """-> list of ('text', s) / ('action', s) with trim markers applied."""
    out = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1) == "-":
            text = text.rstrip()
        out.append(["text", text])
        out.append(["action", m.group(2), m.group(3) == "-"])
        pos = m.end()
    out.append(["text", src[pos:]])
    # apply right-trim markers to the following text
    for i, tok in enumerate(out):
        if tok[0] == "action" and tok[2] and i + 1 < len(out):
            out[i + 1][1] = out[i + 1][1].lstrip()
    return [(t[0], t[1]) for t in out]


def _parse(tokens, i=0, stop=("end",)):
    """Parse into a tree: list of nodes; returns (nodes, index, terminator)."""
    nodes = []
    while i < len(tokens):
        kind, val = tokens[i]
        if kind == "text":
            if val:
                nodes.append(("text", val))
            i += 1
            continue
        if val.startswith("/*"):
            i += 1
            continue
        word = val.split(None, 1)[0] if val else ""
        if word in stop or (word == "else" and "else" in stop):
            return nodes, i, val
        if word in ("if", "with", "range"):
            cond = val[len(word):].strip()
            body, i, term = _parse(tokens, i + 1, stop=("end", "else"))
            branches = [(cond, body)]
            else_body = []
            while term.startswith("else"):
                rest = term[4:].strip()
                if rest.startswith("if "):
                    b, i, term = _parse(tokens, i + 1, stop=("end", "else"))
                    branches.append((rest[3:].strip(), b))
                else:
                    else_body, i, term = _parse(tokens, i + 1, stop=("end",))
            nodes.append((word, branches, else_body))
            i += 1
            continue
        if word == "define":
            name = shlex.split(val[len("define"):].strip())[0]
            body, i, _ = _parse(tokens, i + 1, stop=("end",))
            nodes.append(("define", name, body))
            i += 1
            continue
        nodes.append(("expr", val))
        i += 1
    return nodes, i, None


def _to_yaml(v) -> str:
    if v is None:
        return "null"
    if isinstance(v, (dict, list)):
        if not v:
            return "{}" if isinstance(v, dict) else "[]"
        return yaml.safe_dump(v, sort_keys=False, default_flow_style=False).rstrip("\n")
    return yaml.safe_dump(v).rstrip("\n").removesuffix("\n...").rstrip("\n")


def _truthy(v) -> bool:
    return bool(v) and v not in ("false", 0)


class Renderer:
    def __init__(self, chart_dir: str, values: dict, release_name: str = "gpu-operator",
                 namespace: str = "gpu-operator-resources"):
        self.chart_dir = chart_dir
        with open(os.path.join(chart_dir, "Chart.yaml")) as f:
            self.chart = yaml.load(f, Loader=_Loader)
        self.values = values
        self.release = {"Name": release_name, "Namespace": namespace, "Service": "Helm", "IsInstall": True}
        self.defines: dict[str, list] = {}

    # ------------------------------------------------------------- evaluation
    def _lookup(self, path: str, dot):
        root = {"Values": self.values, "Release": self.release,
                "Chart": {"Name": self.chart.get("name"), "Version": self.chart.get("version"),
                          "AppVersion": self.chart.get("appVersion")}}
        if path == ".":
            return dot
        if path.startswith("$."):
            cur, parts = root, path[2:].split(".")
        elif path.startswith(".Values") or path.startswith(".Release") or path.startswith(".Chart"):
            cur, parts = root, path[1:].split(".")
        else:
            cur, parts = dot, path[1:].split(".")
        for p in parts:
            if not p:
                continue
            cur = cur.get(p) if isinstance(cur, dict) else None
        return cur

    def _atom(self, tok: str, dot):
        if tok.startswith('"') and tok.endswith('"'):
            return tok[1:-1].encode().decode("unicode_escape")
        if tok in ("true", "false"):
            return tok == "true"
        if re.fullmatch(r"-?\d+", tok):
            return int(tok)
        if tok.startswith("."):
            return self._lookup(tok, dot)
        if tok.startswith("$."):
            return self._lookup(tok, dot)
        if tok == "nil":
            return None
        raise TemplateError(f"cannot evaluate {tok!r}")

    def _split_args(self, s: str) -> list[str]:
        toks, cur, depth, q = [], "", 0, False
        for ch in s:
            if ch == '"' and not cur.endswith("\\"):
                q = not q
            if not q and ch == "(":
                depth += 1
            if not q and ch == ")":
                depth -= 1
            if ch.isspace() and not q and depth == 0:
                if cur:
                    toks.append(cur)
                cur = ""
            else:
                cur += ch
        if cur:
            toks.append(cur)
        return toks

    def _call(self, fn: str, args: list, dot):
        if fn == "toYaml":
            return _to_yaml(args[0])
        if fn == "nindent":
            n, s = args
            return "\n" + "\n".join((" " * n + line) if line else line for line in str(s).split("\n"))
        if fn == "indent":
            n, s = args
            return "\n".join((" " * n + line) if line else line for line in str(s).split("\n"))
        if fn == "quote":
            return '"' + str("" if args[0] is None else args[0]).replace('"', '\\"') + '"'
        if fn == "default":
            d, v = args
            return v if _truthy(v) else d  # Helm semantics: false / 0 / "" are "empty"
        if fn == "not":
            return not _truthy(args[0])
        if fn == "and":
            return all(_truthy(a) for a in args)
        if fn == "or":
            return next((a for a in args if _truthy(a)), args[-1] if args else None)
        if fn == "eq":
            return args[0] == args[1]
        if fn == "ne":
            return args[0] != args[1]
        if fn == "printf":
            fmt = args[0].replace("%d", "%s")
            return fmt % tuple(args[1:])
        if fn == "trunc":
            return str(args[1])[: args[0]]
        if fn == "trimSuffix":
            return str(args[1]).removesuffix(args[0])
        if fn == "include":
            return self._render_nodes(self.defines[args[0]], args[1] if len(args) > 1 else dot)
        raise TemplateError(f"unsupported function {fn}")

    def _eval_cmd(self, cmd: str, dot, piped=None, has_pipe=False):
        toks = self._split_args(cmd.strip())
        if not toks:
            raise TemplateError("empty command")
        head = toks[0]
        args = [self._eval(t, dot) for t in toks[1:]]
        if has_pipe:
            args.append(piped)
        if head.startswith(".") or head.startswith('"') or head.startswith("$") or re.fullmatch(r"-?\d+|true|false", head):
            if len(toks) > 1 or has_pipe:
                raise TemplateError(f"cannot apply arguments to {head}")
            return self._atom(head, dot)
        return self._call(head, args, dot)

    def _eval(self, expr: str, dot):
        expr = expr.strip()
        if expr.startswith("(") and expr.endswith(")"):
            return self._eval_pipeline(expr[1:-1], dot)
        return self._atom(expr, dot) if not re.match(r"^[A-Za-z]", expr) else self._eval_cmd(expr, dot)

    def _eval_pipeline(self, expr: str, dot):
        parts, cur, depth, q = [], "", 0, False
        for ch in expr:
            if ch == '"':
                q = not q
            if not q and ch == "(":
                depth += 1
            if not q and ch == ")":
                depth -= 1
            if ch == "|" and not q and depth == 0:
                parts.append(cur)
                cur = ""
            else:
                cur += ch
        parts.append(cur)
        val = self._eval_cmd(parts[0], dot)
        for p in parts[1:]:
            val = self._eval_cmd(p, dot, val, True)
        return val

    # -------------------------------------------------------------- rendering
    def _render_nodes(self, nodes, dot) -> str:
        out = []
        for n in nodes:
            kind = n[0]
            if kind == "text":
                out.append(n[1])
            elif kind == "expr":
                v = self._eval_pipeline(n[1], dot)
                out.append("" if v is None else (str(v).lower() if isinstance(v, bool) else str(v)))
            elif kind == "define":
                self.defines[n[1]] = n[2]
            elif kind in ("if", "with"):
                branches, else_body = n[1], n[2]
                done = False
                for cond, body in branches:
                    v = self._eval_pipeline(cond, dot)
                    if _truthy(v):
                        out.append(self._render_nodes(body, v if kind == "with" else dot))
                        done = True
                        break
                if not done:
                    out.append(self._render_nodes(else_body, dot))
            elif kind == "range":
                (cond, body), = n[1][:1]
                seq = self._eval_pipeline(cond, dot) or []
                items = seq.items() if isinstance(seq, dict) else enumerate(seq)
                for _, item in items:
                    out.append(self._render_nodes(body, item))
        return "".join(out)

    def render_file(self, path: str) -> str:
        with open(path) as f:
            nodes, _, _ = _parse(_tokenize(f.read()))
        return self._render_nodes(nodes, {"Values": self.values})

    def render(self) -> dict[str, str]:
        tdir = os.path.join(self.chart_dir, "templates")
        for fn in sorted(os.listdir(tdir)):
            if fn.endswith(".tpl"):
                self.render_file(os.path.join(tdir, fn))  # collects defines
        out = {}
        for fn in sorted(os.listdir(tdir)):
            if fn.endswith((".yaml", ".yml")):
                out[fn] = self.render_file(os.path.join(tdir, fn))
        return out


def chart_values(overrides: dict | None = None, set_flags: list[str] | None = None,
                 chart_dir: str = CHART_DIR) -> dict:
    with open(os.path.join(chart_dir, "values.yaml")) as f:
        values = yaml.load(f, Loader=_Loader) or {}
    if overrides:
        values = deep_merge(values, overrides)
    if set_flags:
        values = deep_merge(values, parse_set_flags(set_flags))
    return values


def render_chart(values: dict | None = None, set_flags: list[str] | None = None, release_name: str = "gpu-operator",
                 namespace: str = "gpu-operator-resources", chart_dir: str = CHART_DIR) -> list[dict]:
    """Render the chart into Kubernetes objects (CRDs from ``crds/`` first)."""
    vals = chart_values(values, set_flags, chart_dir)
    docs: list[dict] = []
    crd_dir = os.path.join(chart_dir, "crds")
    for fn in sorted(os.listdir(crd_dir)):
        with open(os.path.join(crd_dir, fn)) as f:
            docs += [d for d in yaml.load_all(f, Loader=_Loader) if d]
    for _, text in Renderer(chart_dir, vals, release_name, namespace).render().items():
        docs += [d for d in yaml.load_all(text, Loader=_Loader) if d]
    return docs


def load_crd(chart_dir: str = CHART_DIR) -> dict:
    with open(os.path.join(chart_dir, "crds", "amd.com_clusterpolicies.yaml")) as f:
        return yaml.load(f, Loader=_Loader)
