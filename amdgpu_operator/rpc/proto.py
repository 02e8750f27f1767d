"""Protocol-buffer messages from a compact schema, in plain Python.

The kubelet APIs the operator speaks (device plugin ``v1beta1``, pod
resources ``v1``; deviceplugin/api.py; /root/reference/README.md:122,211,220) are a few flat messages of strings,
bools, integers, nested messages and one string map.  Encoding them needs no
descriptor pool: this module builds message classes straight from the
``{"Msg": [(field, number, type, label)]}`` schema and writes/reads the
proto3 wire format (varint / length-delimited / fixed64 / fixed32, packed or
unpacked repeated scalars, map entries as ``{1: key, 2: value}``, unknown
fields skipped).  Importing google.protobuf and building the descriptors cost
each operand process ~25 ms of start-up (the device plugin and the validator
are on the time-to-Ready critical path); this module imports in under 1 ms.
tests/test_rpc.py checks every message against google.protobuf's own codec
(deviceplugin/protodef.py) in both directions.

The subset of the protobuf Python API the operator uses is kept: keyword
constructors, attribute access, ``repeated.add(**kw)`` / ``append`` /
``extend``, map fields as dicts, sub-messages created on first access
(``req.options.flag = True``), ``SerializeToString()`` and ``FromString()``.
"""

from __future__ import annotations

import struct

VARINT, I64, LEN, I32 = 0, 1, 2, 5

# scalar type -> (wire type, default)
SCALARS = {
    "string": (LEN, ""),
    "bytes": (LEN, b""),
    "bool": (VARINT, False),
    "int32": (VARINT, 0),
    "int64": (VARINT, 0),
    "uint32": (VARINT, 0),
    "uint64": (VARINT, 0),
    "double": (I64, 0.0),
    "float": (I32, 0.0),
}


class DecodeError(ValueError):
    pass


def put_varint(out: bytearray, v: int) -> None:
    v &= (1 << 64) - 1  # negative int32/int64: ten-byte two's complement, as protoc writes it
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)


def get_varint(buf, pos: int) -> tuple[int, int]:
    v = shift = 0
    n = len(buf)
    while True:
        if pos >= n:
            raise DecodeError("truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7
        if shift >= 70:
            raise DecodeError("varint too long")


def _scalar_from_varint(ftype: str, v: int):
    if ftype == "bool":
        return v != 0
    if ftype == "int64":
        return v - (1 << 64) if v >= 1 << 63 else v
    if ftype == "int32":
        v &= 0xFFFFFFFF
        return v - (1 << 32) if v >= 1 << 31 else v
    if ftype == "uint32":
        return v & 0xFFFFFFFF
    return v


def _put_scalar(out: bytearray, ftype: str, v) -> None:
    wt = SCALARS[ftype][0]
    if wt == VARINT:
        put_varint(out, int(v))
    elif wt == LEN:
        b = v.encode() if isinstance(v, str) else bytes(v)
        put_varint(out, len(b))
        out += b
    elif wt == I64:
        out += struct.pack("<d", float(v))
    else:
        out += struct.pack("<f", float(v))


class Field:
    __slots__ = ("name", "number", "type", "repeated", "map_types", "msg_cls")

    def __init__(self, name: str, number: int, ftype: str, label: str):
        self.name, self.number = name, number
        self.repeated = label == "rep"
        self.map_types = None
        self.msg_cls = None  # resolved after every class of the file exists
        if ftype.startswith("map<"):
            k, v = ftype[4:-1].split(",")
            self.map_types = (k.strip(), v.strip())
            self.repeated = True
        self.type = ftype

    @property
    def is_message(self) -> bool:
        return self.map_types is None and self.type not in SCALARS


class RepeatedMessage(list):
    """A repeated message field: a list with protobuf's ``add(**kw)``."""

    __slots__ = ("_cls",)

    def __init__(self, cls, items=()):
        super().__init__()
        self._cls = cls
        self.extend(items)

    def add(self, **kw):
        m = self._cls(**kw)
        super().append(m)
        return m

    def append(self, m) -> None:
        super().append(m if isinstance(m, Message) else self._cls(**m))

    def extend(self, items) -> None:
        for m in items:
            self.append(m)


class Message:
    """Base of the generated classes (see :func:`build_file`)."""

    FIELDS: tuple = ()
    BY_NAME: dict = {}
    BY_NUMBER: dict = {}
    __slots__ = ("_values", "_present")

    def __init__(self, **kw):
        object.__setattr__(self, "_values", {})
        object.__setattr__(self, "_present", set())  # message fields set explicitly (or seen on the wire)
        for k, v in kw.items():
            setattr(self, k, v)

    # ------------------------------------------------------------ attributes
    def _default(self, f: Field):
        if f.map_types is not None:
            return {}
        if f.repeated:
            return RepeatedMessage(f.msg_cls) if f.is_message else []
        if f.is_message:
            return f.msg_cls()
        return SCALARS[f.type][1]

    def __getattr__(self, name):
        f = type(self).BY_NAME.get(name)
        if f is None:
            raise AttributeError(f"{type(self).__name__} has no field {name!r}")
        vals = self._values
        if name not in vals:
            vals[name] = self._default(f)
        return vals[name]

    def __setattr__(self, name, value):
        f = type(self).BY_NAME.get(name)
        if f is None:
            raise AttributeError(f"{type(self).__name__} has no field {name!r}")
        if f.map_types is not None:
            value = dict(value)
        elif f.repeated:
            value = RepeatedMessage(f.msg_cls, value) if f.is_message else list(value)
        elif f.is_message:
            if isinstance(value, dict):
                value = f.msg_cls(**value)
            elif not isinstance(value, f.msg_cls):
                raise TypeError(f"{name}: expected {f.msg_cls.__name__}, got {type(value).__name__}")
            self._present.add(name)
        self._values[name] = value

    def HasField(self, name: str) -> bool:  # noqa: N802 - protobuf's name
        f = type(self).BY_NAME[name]
        if not f.is_message or f.repeated:
            raise ValueError(f"{name} is not a singular message field")
        m = self._values.get(name)
        return m is not None and (name in self._present or m._nonempty())

    def _nonempty(self) -> bool:
        for f in type(self).FIELDS:
            v = self._values.get(f.name)
            if v is None:
                continue
            if f.is_message and not f.repeated:
                if f.name in self._present or v._nonempty():
                    return True
            elif v:
                return True
        return False

    def __eq__(self, other):
        return type(other) is type(self) and self.SerializeToString() == other.SerializeToString()

    def __repr__(self):
        parts = []
        for f in type(self).FIELDS:
            v = self._values.get(f.name)
            if v is None or (not v and not (f.is_message and f.name in self._present)):
                continue
            parts.append(f"{f.name}={v!r}")
        return f"{type(self).__name__}({', '.join(parts)})"

    # -------------------------------------------------------------- encoding
    def _encode(self, out: bytearray) -> None:
        for f in type(self).FIELDS:  # field-number order, as protoc writes
            v = self._values.get(f.name)
            if v is None:
                continue
            num = f.number
            if f.map_types is not None:
                kt, vt = f.map_types
                for k, x in v.items():
                    entry = bytearray()
                    put_varint(entry, (1 << 3) | SCALARS[kt][0])
                    _put_scalar(entry, kt, k)
                    put_varint(entry, (2 << 3) | SCALARS[vt][0])
                    _put_scalar(entry, vt, x)
                    put_varint(out, (num << 3) | LEN)
                    put_varint(out, len(entry))
                    out += entry
            elif f.is_message:
                for m in (v if f.repeated else (v,)):
                    sub = bytearray()
                    m._encode(sub)
                    if not f.repeated and not sub and f.name not in self._present:
                        continue  # an untouched sub-message is absent
                    put_varint(out, (num << 3) | LEN)
                    put_varint(out, len(sub))
                    out += sub
            elif f.repeated:
                if not v:
                    continue
                wt = SCALARS[f.type][0]
                if wt == LEN:  # strings / bytes are never packed
                    for x in v:
                        put_varint(out, (num << 3) | LEN)
                        _put_scalar(out, f.type, x)
                else:  # proto3 packs repeated numeric fields
                    packed = bytearray()
                    for x in v:
                        _put_scalar(packed, f.type, x)
                    put_varint(out, (num << 3) | LEN)
                    put_varint(out, len(packed))
                    out += packed
            else:
                if v == SCALARS[f.type][1]:
                    continue  # proto3: default values are not written
                put_varint(out, (num << 3) | SCALARS[f.type][0])
                _put_scalar(out, f.type, v)

    def SerializeToString(self) -> bytes:  # noqa: N802 - protobuf's name
        out = bytearray()
        self._encode(out)
        return bytes(out)

    @classmethod
    def FromString(cls, data) -> "Message":  # noqa: N802 - protobuf's name
        m = cls()
        m._decode(memoryview(bytes(data)), 0, len(data))
        return m

    def _decode(self, buf, pos: int, end: int) -> None:
        by_num = type(self).BY_NUMBER
        vals = self._values
        while pos < end:
            key, pos = get_varint(buf, pos)
            num, wt = key >> 3, key & 7
            if num == 0:
                raise DecodeError("field number 0")
            f = by_num.get(num)
            if wt == VARINT:
                v, pos = get_varint(buf, pos)
                raw = None
            elif wt == LEN:
                n, pos = get_varint(buf, pos)
                if pos + n > end:
                    raise DecodeError("truncated length-delimited field")
                raw, pos = (pos, pos + n), pos + n
            elif wt == I64:
                if pos + 8 > end:
                    raise DecodeError("truncated fixed64")
                raw, v, pos = None, bytes(buf[pos:pos + 8]), pos + 8
            elif wt == I32:
                if pos + 4 > end:
                    raise DecodeError("truncated fixed32")
                raw, v, pos = None, bytes(buf[pos:pos + 4]), pos + 4
            else:
                raise DecodeError(f"unsupported wire type {wt}")
            if f is None:
                continue  # unknown field: skipped
            if f.map_types is not None:
                if raw is None:
                    raise DecodeError(f"{f.name}: map entry is not length-delimited")
                k, x = _decode_entry(buf, raw[0], raw[1], f.map_types)
                self.__getattr__(f.name)[k] = x
            elif f.is_message:
                if raw is None:
                    raise DecodeError(f"{f.name}: message is not length-delimited")
                if f.repeated:
                    sub = f.msg_cls()
                    sub._decode(buf, raw[0], raw[1])
                    self.__getattr__(f.name).append(sub)
                else:  # a repeated occurrence of a singular message merges into it
                    sub = vals.get(f.name) or f.msg_cls()
                    sub._decode(buf, raw[0], raw[1])
                    vals[f.name] = sub
                    self._present.add(f.name)
            else:
                x = _decode_scalar(buf, f.type, wt, v if raw is None else raw, f.repeated)
                if f.repeated:
                    self.__getattr__(f.name).extend(x)
                else:
                    vals[f.name] = x


def _decode_one(buf, ftype: str, wt: int, v):
    want = SCALARS[ftype][0]
    if wt != want:
        raise DecodeError(f"{ftype}: wire type {wt}, expected {want}")
    if wt == VARINT:
        return _scalar_from_varint(ftype, v)
    if wt == LEN:
        b = bytes(buf[v[0]:v[1]])
        if ftype == "string":
            try:
                return b.decode()
            except UnicodeDecodeError as e:
                raise DecodeError(f"string field is not UTF-8: {e}") from None
        return b
    if wt == I64:
        return struct.unpack("<d", v)[0]
    return struct.unpack("<f", v)[0]


def _decode_scalar(buf, ftype: str, wt: int, v, repeated: bool):
    """One scalar, or (repeated) the list one occurrence carries - packed
    numeric runs included."""
    if not repeated:
        return _decode_one(buf, ftype, wt, v)
    if wt == LEN and SCALARS[ftype][0] != LEN:  # packed run
        out, pos, end = [], v[0], v[1]
        want = SCALARS[ftype][0]
        while pos < end:
            if want == VARINT:
                x, pos = get_varint(buf, pos)
                out.append(_scalar_from_varint(ftype, x))
            else:
                size = 8 if want == I64 else 4
                if pos + size > end:
                    raise DecodeError("truncated packed field")
                out.append(_decode_one(buf, ftype, want, bytes(buf[pos:pos + size])))
                pos += size
        return out
    return [_decode_one(buf, ftype, wt, v)]


def _decode_entry(buf, pos: int, end: int, types: tuple[str, str]):
    kt, vt = types
    k, x = SCALARS[kt][1], SCALARS[vt][1]
    while pos < end:
        key, pos = get_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if wt == VARINT:
            v, pos = get_varint(buf, pos)
        elif wt == LEN:
            n, pos = get_varint(buf, pos)
            v, pos = (pos, pos + n), pos + n
            if pos > end:
                raise DecodeError("truncated map entry")
        elif wt in (I64, I32):
            size = 8 if wt == I64 else 4
            v, pos = bytes(buf[pos:pos + size]), pos + size
        else:
            raise DecodeError(f"unsupported wire type {wt}")
        if num == 1:
            k = _decode_one(buf, kt, wt, v)
        elif num == 2:
            x = _decode_one(buf, vt, wt, v)
    return k, x


def build_file(package: str, messages: dict[str, list[tuple]]) -> dict[str, type]:
    """``{"Msg": [(field, number, type, label)]}`` -> ``{"Msg": class}``.

    ``type``: a scalar name (:data:`SCALARS`), another message of the same
    schema, or ``"map<string,string>"``; ``label``: ``"opt"`` or ``"rep"``."""
    classes: dict[str, type] = {}
    for name, fields in messages.items():
        fs = tuple(sorted((Field(*f) for f in fields), key=lambda f: f.number))
        classes[name] = type(name, (Message,), {
            "__slots__": (), "__module__": f"{__name__}.{package}", "FIELDS": fs,
            "BY_NAME": {f.name: f for f in fs}, "BY_NUMBER": {f.number: f for f in fs}})
    for cls in classes.values():
        for f in cls.FIELDS:
            if f.is_message:
                if f.type not in classes:
                    raise ValueError(f"{cls.__name__}.{f.name}: unknown message type {f.type}")
                f.msg_cls = classes[f.type]
    return classes
