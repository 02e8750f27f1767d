"""Operand command lines parsed without importing argparse.

Every operand container starts as ``python3 -S -m amdgpu_operator <cmd>``,
and its start is on the bring-up's critical path (the driver container's,
then the validator's).  Importing argparse costs a fresh interpreter 7.8 ms
on the MI355X box (``profiles/r5_ttr/startup``), more than parsing the
command line takes.

:class:`Spec` records the sub-commands and arguments through argparse's own
method names (``add_subparsers`` / ``add_parser`` / ``add_argument``), so
``cli/operands.py`` declares the command line once.  :meth:`Spec.parse`
handles the forms the operator renders: exact long options, ``--opt value``
and ``--opt=value``, ``store_true`` flags, typed values, choices and
positionals.  For anything else it builds the argparse parser from the same
record and lets argparse parse: help, errors, abbreviations, negative numbers
as values.  Its result is then argparse's own, so the fast path never
accepts a command line that argparse would parse differently.
``tests/test_argspec.py`` compares the two on every command the operator
renders.
"""

from __future__ import annotations

from types import SimpleNamespace

_BAD = object()


class _Command:
    def __init__(self) -> None:
        self.calls: list[tuple[tuple, dict]] = []
        self.options: dict[str, tuple[str, dict]] = {}
        self.positionals: list[tuple[str, dict]] = []

    def add_argument(self, *names: str, **kw) -> None:
        self.calls.append((names, kw))
        if names[0].startswith("-"):
            long = next((n for n in names if n.startswith("--")), names[0])
            dest = kw.get("dest") or long.lstrip("-").replace("-", "_")
            for n in names:
                self.options[n] = (dest, kw)
        else:
            self.positionals.append((names[0], kw))


class _Subcommands:
    def __init__(self, spec: "Spec") -> None:
        self.spec = spec

    def add_parser(self, name: str, **kw) -> _Command:
        cmd = _Command()
        self.spec.commands[name] = (cmd, kw)
        return cmd


def _convert(value: str, kw: dict):
    t = kw.get("type")
    if t is not None:
        try:
            value = t(value)
        except (TypeError, ValueError):
            return _BAD
    if "choices" in kw and value not in kw["choices"]:
        return _BAD
    return value


class Spec:
    """A parser declaration with argparse's interface (the subset above)."""

    def __init__(self, **parser_kw) -> None:
        self.parser_kw = parser_kw
        self.sub_kw: dict = {}
        self.commands: dict[str, tuple[_Command, dict]] = {}

    def add_subparsers(self, **kw) -> _Subcommands:
        self.sub_kw = kw
        return _Subcommands(self)

    def argparse(self):
        """The same declaration as an ``argparse.ArgumentParser``."""
        import argparse

        p = argparse.ArgumentParser(**self.parser_kw)
        sub = p.add_subparsers(**self.sub_kw)
        for name, (cmd, kw) in self.commands.items():
            sp = sub.add_parser(name, **kw)
            for names, akw in cmd.calls:
                sp.add_argument(*names, **akw)
        return p

    def parse(self, argv: list[str]):
        ns = self._fast(list(argv))
        return ns if ns is not None else self.argparse().parse_args(argv)

    def _fast(self, argv: list[str]):
        if not argv or argv[0] not in self.commands or not self.sub_kw.get("dest"):
            return None
        cmd, _ = self.commands[argv[0]]
        values: dict = {self.sub_kw["dest"]: argv[0]}
        for names, kw in cmd.calls:
            if not names[0].startswith("-"):
                continue
            dest, _ = cmd.options[names[0]]
            action = kw.get("action")
            if action == "store_true":
                values[dest] = kw.get("default", False)
            elif action is not None or kw.get("nargs") is not None:
                return None  # not a form this parser handles
            else:
                d = kw.get("default")
                if isinstance(d, str) and kw.get("type") is not None:
                    d = _convert(d, {"type": kw["type"]})  # argparse converts string defaults
                    if d is _BAD:
                        return None
                values[dest] = d
        positionals: list[str] = []
        i = 1
        while i < len(argv):
            tok = argv[i]
            if not tok.startswith("-"):
                positionals.append(tok)
                i += 1
                continue
            if not tok.startswith("--") or tok == "--":
                return None  # -h, short options, negative numbers, "--"
            name, eq, value = tok.partition("=")
            opt = cmd.options.get(name)
            if opt is None:
                return None  # --help, an abbreviation, an unknown option: argparse decides
            dest, kw = opt
            if kw.get("action") == "store_true":
                if eq:
                    return None
                values[dest] = True
                i += 1
                continue
            if not eq:
                if i + 1 >= len(argv) or argv[i + 1].startswith("-"):
                    return None
                value = argv[i + 1]
                i += 2
            else:
                i += 1
            value = _convert(value, kw)
            if value is _BAD:
                return None
            values[dest] = value
        if len(positionals) != len(cmd.positionals):
            return None
        for (name, kw), tok in zip(cmd.positionals, positionals):
            value = _convert(tok, kw)
            if value is _BAD:
                return None
            values[name] = value
        return SimpleNamespace(**values)
