"""Dataclass-shaped value classes without the ``dataclasses`` module.

``import dataclasses`` imports ``inspect`` (and with it ``ast``, ``dis``,
``tokenize``): 16 ms of a fresh interpreter on the MI355X box
(``profiles/r5_ttr/startup``), paid by every operand process the bring-up
starts - the driver container, the validator, the device plugin - before
its first useful line.  The few classes on those start-up paths (kube
resource types, the node environment, the topology records) use this
instead: ``__init__`` in field order with defaults and ``field(default_factory=...)``,
``__repr__``, ``__eq__``, ``frozen=True`` (immutable, hashable), :func:`asdict` and :func:`replace`.
"""

from __future__ import annotations

import copy

_MISSING = object()


class field:  # noqa: N801 - the dataclasses name, for the same use
    """A default built per instance (``field(default_factory=dict)``)."""

    __slots__ = ("default_factory",)

    def __init__(self, default_factory):
        self.default_factory = default_factory


def record(cls=None, *, frozen: bool = False):
    def wrap(cls):
        names = list(cls.__dict__.get("__annotations__", {}))
        ns = {"_MISSING": _MISSING, "_set": object.__setattr__}
        args, body = [], []
        for n in names:
            if n in cls.__dict__:
                d = cls.__dict__[n]
                if isinstance(d, field):
                    ns[f"_f_{n}"] = d.default_factory
                    args.append(f"{n}=_MISSING")
                    val = f"_f_{n}() if {n} is _MISSING else {n}"
                    delattr(cls, n)
                else:
                    ns[f"_d_{n}"] = d
                    args.append(f"{n}=_d_{n}")
                    val = n
            else:
                args.append(n)
                val = n
            body.append(f"    _set(self, {n!r}, {val})")
        src = f"def __init__(self{''.join(', ' + a for a in args)}):\n" + ("\n".join(body) or "    pass")
        exec(src, ns)  # noqa: S102 - generated from the class's own field names
        ns["__init__"].__qualname__ = f"{cls.__qualname__}.__init__"
        cls.__init__ = ns["__init__"]
        cls.__record_fields__ = tuple(names)

        def __repr__(self):
            return f"{type(self).__name__}(" + ", ".join(f"{n}={getattr(self, n)!r}" for n in names) + ")"

        def __eq__(self, other):
            if other.__class__ is not self.__class__:
                return NotImplemented
            return all(getattr(self, n) == getattr(other, n) for n in names)

        cls.__repr__ = __repr__
        cls.__eq__ = __eq__
        if frozen:
            def __setattr__(self, n, v):
                raise AttributeError(f"cannot assign to field {n!r} of a frozen {type(self).__name__}")

            cls.__setattr__ = __setattr__
            cls.__delattr__ = __setattr__
            cls.__hash__ = lambda self: hash(tuple(getattr(self, n) for n in names))
        else:
            cls.__hash__ = None  # mutable and compared by value: unhashable, like a dataclass
        return cls

    return wrap(cls) if cls is not None else wrap


def replace(obj, **changes):
    """A copy with some fields changed (``dataclasses.replace``)."""
    return type(obj)(**{n: changes.get(n, getattr(obj, n)) for n in type(obj).__record_fields__})


def fields_of(obj) -> tuple[str, ...]:
    return type(obj).__record_fields__


def asdict(obj):
    """Recursive copy into plain dicts / lists (``dataclasses.asdict``)."""
    if hasattr(type(obj), "__record_fields__"):
        return {n: asdict(getattr(obj, n)) for n in type(obj).__record_fields__}
    if isinstance(obj, (list, tuple)):
        return type(obj)(asdict(v) for v in obj)
    if isinstance(obj, dict):
        return {asdict(k): asdict(v) for k, v in obj.items()}
    return copy.deepcopy(obj)
