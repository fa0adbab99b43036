"""Message types and service plumbing of the gRPC API (api/proto/*.proto).

The image has the grpc and protobuf runtimes but no protoc, so the .proto
files themselves are the source: `load(path)` reads the proto3 subset they use
(messages with scalar, message, enum and repeated fields; nested enums;
services of unary methods), builds a FileDescriptorProto, and returns the
message classes and the service's method table.  A Go build would feed the
same files to protoc (Makefile:82-85 of the reference).
"""
from __future__ import annotations

import os
import re

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PROTO_DIR = os.path.join(ROOT, "api", "proto")

_F = descriptor_pb2.FieldDescriptorProto
_SCALARS = {
    "double": _F.TYPE_DOUBLE, "float": _F.TYPE_FLOAT, "int64": _F.TYPE_INT64, "uint64": _F.TYPE_UINT64,
    "int32": _F.TYPE_INT32, "uint32": _F.TYPE_UINT32, "bool": _F.TYPE_BOOL, "string": _F.TYPE_STRING,
    "bytes": _F.TYPE_BYTES, "sint64": _F.TYPE_SINT64, "sint32": _F.TYPE_SINT32,
}


def _tokens(text: str):
    text = re.sub(r"//[^\n]*", "", text)
    return re.findall(r'"[^"]*"|[A-Za-z_][\w.]*|\d+|[{}();=<>,\[\]]', text)


class _Parser:
    def __init__(self, text):
        self.t = _tokens(text)
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        if want is not None and tok != want:
            raise ValueError(f"proto: expected {want!r}, got {tok!r} (token {self.i})")
        self.i += 1
        return tok


def parse(text: str, name: str) -> tuple[descriptor_pb2.FileDescriptorProto, dict]:
    """FileDescriptorProto + {service: [(method, input, output)]} of a .proto"""
    p = _Parser(text)
    fdp = descriptor_pb2.FileDescriptorProto(name=name, syntax="proto3")
    services = {}
    enums_nested = {}   # message -> names of its nested enums

    def parse_enum(container):
        ename = p.take()
        e = container.add(name=ename)
        p.take("{")
        while p.peek() != "}":
            vname = p.take()
            p.take("=")
            num = int(p.take())
            p.take(";")
            e.value.add(name=vname, number=num)
        p.take("}")
        return ename

    def parse_message(container):
        mname = p.take()
        msg = container.add(name=mname)
        p.take("{")
        nested = []
        while p.peek() != "}":
            tok = p.take()
            if tok == "enum":
                nested.append(parse_enum(msg.enum_type))
                continue
            label = _F.LABEL_OPTIONAL
            if tok == "repeated":
                label = _F.LABEL_REPEATED
                tok = p.take()
            fname = p.take()
            p.take("=")
            num = int(p.take())
            p.take(";")
            f = msg.field.add(name=fname, number=num, label=label, json_name=fname)
            if tok in _SCALARS:
                f.type = _SCALARS[tok]
            else:
                f.type_name = tok   # resolved below (message or enum)
        p.take("}")
        enums_nested[mname] = nested
        return msg

    while p.peek() is not None:
        tok = p.take()
        if tok == "syntax":
            p.take("=")
            p.take()
            p.take(";")
        elif tok == "package":
            fdp.package = p.take()
            p.take(";")
        elif tok == "option":
            while p.take() != ";":
                pass
        elif tok == "message":
            parse_message(fdp.message_type)
        elif tok == "enum":
            parse_enum(fdp.enum_type)
        elif tok == "service":
            sname = p.take()
            p.take("{")
            methods = []
            sd = fdp.service.add(name=sname)
            while p.peek() != "}":
                p.take("rpc")
                mname = p.take()
                p.take("(")
                inp = p.take()
                p.take(")")
                p.take("returns")
                p.take("(")
                out = p.take()
                p.take(")")
                p.take(";")
                pre = "." + fdp.package + "."
                sd.method.add(name=mname, input_type=pre + inp, output_type=pre + out)
                methods.append((mname, inp, out))
            p.take("}")
            services[sname] = methods
        else:
            raise ValueError(f"proto: unexpected {tok!r}")
    # resolve field type names: nested enum, top-level message or enum
    top_msgs = {m.name for m in fdp.message_type}
    top_enums = {e.name for e in fdp.enum_type}
    pre = "." + fdp.package + "."
    for m in fdp.message_type:
        for f in m.field:
            if not f.type_name:
                continue
            n = f.type_name
            if n in enums_nested.get(m.name, []):
                f.type, f.type_name = _F.TYPE_ENUM, pre + m.name + "." + n
            elif n in top_msgs:
                f.type, f.type_name = _F.TYPE_MESSAGE, pre + n
            elif n in top_enums:
                f.type, f.type_name = _F.TYPE_ENUM, pre + n
            else:
                raise ValueError(f"proto: unknown type {n!r} in {m.name}")
    return fdp, services


class Api:
    """Message classes (attributes by message name) and service method tables
    of one .proto file."""

    def __init__(self, filename: str):
        path = os.path.join(PROTO_DIR, filename)
        fdp, self.services = parse(open(path).read(), filename)
        self.package = fdp.package
        self.fdp = fdp
        pool = descriptor_pool.DescriptorPool()
        pool.Add(fdp)
        for m in fdp.message_type:
            setattr(self, m.name, message_factory.GetMessageClass(pool.FindMessageTypeByName(f"{fdp.package}.{m.name}")))

    def full_service(self, name: str) -> str:
        return f"{self.package}.{name}"


_cache: dict[str, Api] = {}


def api(filename: str = "ratelimiter.proto") -> Api:
    if filename not in _cache:
        _cache[filename] = Api(filename)
    return _cache[filename]


class Stub:
    """Client stub of a service: one callable per method (unary)."""

    def __init__(self, channel, a: Api, service: str):
        for mname, inp, out in a.services[service]:
            setattr(self, mname, channel.unary_unary(
                f"/{a.full_service(service)}/{mname}",
                request_serializer=getattr(a, inp).SerializeToString,
                response_deserializer=getattr(a, out).FromString))


def rate_limiter_stub(channel):
    return Stub(channel, api("ratelimiter.proto"), "RateLimiter")


def health_stub(channel):
    return Stub(channel, api("health.proto"), "Health")
