"""Build protobuf message classes from a compact schema (no ``protoc`` needed).

The build environment has protobuf + grpcio but no ``protoc``/``grpc_tools``
(SURVEY.md §7.1), so the kubelet APIs are declared here as
``FileDescriptorProto`` objects and turned into real message classes through a
private descriptor pool.  The wire format is exactly what protoc would
generate for the same field numbers and types.
"""

from __future__ import annotations

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
_SCALARS = {
    "string": F.TYPE_STRING,
    "bool": F.TYPE_BOOL,
    "int32": F.TYPE_INT32,
    "int64": F.TYPE_INT64,
    "uint32": F.TYPE_UINT32,
    "uint64": F.TYPE_UINT64,
    "bytes": F.TYPE_BYTES,
    "double": F.TYPE_DOUBLE,
}


def _camel(name: str) -> str:
    return "".join(p[:1].upper() + p[1:] for p in name.split("_"))


def build_file(package: str, filename: str, messages: dict[str, list[tuple]], services: dict[str, list[tuple]] | None = None):
    """Create message classes.

    ``messages``: ``{"Msg": [(field, number, type, label), ...]}`` where type is a
    scalar name, another message name, or ``"map<string,T>"`` (T a scalar or a message); label is
    ``"opt"`` or ``"rep"``.
    ``services``: ``{"Svc": [(method, input, output, server_streaming), ...]}``
    (recorded in the descriptor for completeness; gRPC wiring is done with
    generic handlers).
    Returns ``{name: class}``.
    """
    fdp = descriptor_pb2.FileDescriptorProto(name=filename, package=package, syntax="proto3")
    for mname, fields in messages.items():
        m = fdp.message_type.add(name=mname)
        for fname, num, ftype, label in fields:
            f = m.field.add(name=fname, number=num, json_name=fname)
            f.label = F.LABEL_REPEATED if label == "rep" else F.LABEL_OPTIONAL
            if ftype.startswith("map<"):
                kt, vt = ftype[4:-1].split(",")
                entry = m.nested_type.add(name=_camel(fname) + "Entry")
                entry.options.map_entry = True
                entry.field.add(name="key", number=1, type=_SCALARS[kt.strip()], label=F.LABEL_OPTIONAL, json_name="key")
                vt = vt.strip()
                if vt in _SCALARS:
                    entry.field.add(name="value", number=2, type=_SCALARS[vt], label=F.LABEL_OPTIONAL, json_name="value")
                else:  # map<string, Message>
                    entry.field.add(name="value", number=2, type=F.TYPE_MESSAGE, type_name=f".{package}.{vt}",
                                    label=F.LABEL_OPTIONAL, json_name="value")
                f.label = F.LABEL_REPEATED
                f.type = F.TYPE_MESSAGE
                f.type_name = f".{package}.{mname}.{entry.name}"
            elif ftype in _SCALARS:
                f.type = _SCALARS[ftype]
            else:
                f.type = F.TYPE_MESSAGE
                f.type_name = f".{package}.{ftype}"
    for sname, methods in (services or {}).items():
        s = fdp.service.add(name=sname)
        for meth, inp, out, stream in methods:
            s.method.add(name=meth, input_type=f".{package}.{inp}", output_type=f".{package}.{out}",
                         server_streaming=bool(stream))
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    return {name: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{package}.{name}")) for name in messages}, fdp
