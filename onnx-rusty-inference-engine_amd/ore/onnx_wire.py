"""Minimal ONNX protobuf wire-format codec (host tooling, no libprotobuf / no `onnx` package).

Covers the message subset the reference engine touches through `onnx-protobuf 0.2.3`
(`/root/reference/src/inference_engine/utils.rs:14-197`, `model_inference.rs:128-162`):
ModelProto -> GraphProto -> {NodeProto, AttributeProto, TensorProto, ValueInfoProto}.
Field numbers follow `/root/reference/models/onnx.proto` (proto2, package onnx).

Used by the synthetic SqueezeNet-1.0 generator (encoder) and by tests to read the golden
`.pb` tensors (decoder).  The product path parses models in C++
(`csrc/onnx_loader.cpp`); this module never feeds the GPU path directly.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# ----------------------------------------------------------------------------- wire reading


def _varint(buf: bytes, pos: int):
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _fields(buf: bytes):
    """Yield (field_number, wire_type, value) over one message's bytes."""
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _varint(buf, pos)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
        elif wt == 1:
            val = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            val = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            val = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield fno, wt, val


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _packed_varints(val, wt) -> List[int]:
    if wt == 0:
        return [_signed64(val)]
    out, pos = [], 0
    while pos < len(val):
        v, pos = _varint(val, pos)
        out.append(_signed64(v))
    return out


@dataclass
class Tensor:
    name: str = ""
    dims: List[int] = field(default_factory=list)
    data_type: int = 0
    raw_data: bytes = b""
    float_data: List[float] = field(default_factory=list)
    int64_data: List[int] = field(default_factory=list)

    def to_numpy(self) -> np.ndarray:
        """Decode like `get_stored_tensor` (`utils.rs:126-144`): raw_data (LE f32 unless INT64),
        else float_data, else int64_data."""
        if self.raw_data:
            dt = np.int64 if self.data_type == 7 else np.float32
            arr = np.frombuffer(self.raw_data, dtype="<" + np.dtype(dt).str[1:]).astype(dt)
        elif self.float_data:
            arr = np.asarray(self.float_data, dtype=np.float32)
        elif self.int64_data:
            arr = np.asarray(self.int64_data, dtype=np.int64)
        else:
            arr = np.zeros(0, dtype=np.float32)
        if self.dims:
            arr = arr.reshape(self.dims)
        return arr


@dataclass
class Attribute:
    name: str = ""
    type: int = 0
    f: float = 0.0
    i: int = 0
    s: bytes = b""
    ints: List[int] = field(default_factory=list)
    floats: List[float] = field(default_factory=list)


@dataclass
class Node:
    input: List[str] = field(default_factory=list)
    output: List[str] = field(default_factory=list)
    name: str = ""
    op_type: str = ""
    attribute: List[Attribute] = field(default_factory=list)

    def attrs(self) -> Dict[str, Attribute]:
        return {a.name: a for a in self.attribute}


@dataclass
class ValueInfo:
    name: str = ""
    elem_type: int = 0
    shape: List[int] = field(default_factory=list)


@dataclass
class Graph:
    name: str = ""
    node: List[Node] = field(default_factory=list)
    initializer: List[Tensor] = field(default_factory=list)
    input: List[ValueInfo] = field(default_factory=list)
    output: List[ValueInfo] = field(default_factory=list)


@dataclass
class Model:
    ir_version: int = 0
    opset: int = 0
    producer_name: str = ""
    graph: Graph = field(default_factory=Graph)


def decode_tensor(buf: bytes) -> Tensor:
    t = Tensor()
    for fno, wt, val in _fields(buf):
        if fno == 1:
            t.dims.extend(_packed_varints(val, wt))
        elif fno == 2:
            t.data_type = val
        elif fno == 4:
            if wt == 2:
                t.float_data.extend(struct.unpack(f"<{len(val) // 4}f", val))
            else:
                t.float_data.append(struct.unpack("<f", val)[0])
        elif fno == 7:
            t.int64_data.extend(_packed_varints(val, wt))
        elif fno == 8:
            t.name = val.decode()
        elif fno == 9:
            t.raw_data = bytes(val)
    return t


def _decode_attr(buf: bytes) -> Attribute:
    a = Attribute()
    for fno, wt, val in _fields(buf):
        if fno == 1:
            a.name = val.decode()
        elif fno == 20:
            a.type = val
        elif fno == 2:
            a.f = struct.unpack("<f", val)[0]
        elif fno == 3:
            a.i = _signed64(val)
        elif fno == 4:
            a.s = bytes(val)
        elif fno == 8:
            a.ints.extend(_packed_varints(val, wt))
        elif fno == 7:
            if wt == 2:
                a.floats.extend(struct.unpack(f"<{len(val) // 4}f", val))
            else:
                a.floats.append(struct.unpack("<f", val)[0])
    return a


def _decode_node(buf: bytes) -> Node:
    n = Node()
    for fno, wt, val in _fields(buf):
        if fno == 1:
            n.input.append(val.decode())
        elif fno == 2:
            n.output.append(val.decode())
        elif fno == 3:
            n.name = val.decode()
        elif fno == 4:
            n.op_type = val.decode()
        elif fno == 5:
            n.attribute.append(_decode_attr(val))
    return n


def _decode_shape(buf: bytes) -> List[int]:
    dims = []
    for fno, _, val in _fields(buf):
        if fno == 1:
            d = -1
            for f2, _, v2 in _fields(val):
                if f2 == 1:
                    d = _signed64(v2)
            dims.append(d)
    return dims


def _decode_value_info(buf: bytes) -> ValueInfo:
    vi = ValueInfo()
    for fno, _, val in _fields(buf):
        if fno == 1:
            vi.name = val.decode()
        elif fno == 2:
            for f2, _, v2 in _fields(val):
                if f2 == 1:  # tensor_type
                    for f3, _, v3 in _fields(v2):
                        if f3 == 1:
                            vi.elem_type = v3
                        elif f3 == 2:
                            vi.shape = _decode_shape(v3)
    return vi


def _decode_graph(buf: bytes) -> Graph:
    g = Graph()
    for fno, _, val in _fields(buf):
        if fno == 1:
            g.node.append(_decode_node(val))
        elif fno == 2:
            g.name = val.decode()
        elif fno == 5:
            g.initializer.append(decode_tensor(val))
        elif fno == 11:
            g.input.append(_decode_value_info(val))
        elif fno == 12:
            g.output.append(_decode_value_info(val))
    return g


def decode_model(buf: bytes) -> Model:
    m = Model()
    for fno, _, val in _fields(buf):
        if fno == 1:
            m.ir_version = val
        elif fno == 2:
            m.producer_name = val.decode()
        elif fno == 7:
            m.graph = _decode_graph(val)
        elif fno == 8:
            for f2, _, v2 in _fields(val):
                if f2 == 2:
                    m.opset = v2
    return m


def load_model(path) -> Model:
    with open(path, "rb") as f:
        return decode_model(f.read())


def load_tensor(path) -> Tensor:
    with open(path, "rb") as f:
        return decode_tensor(f.read())

# ----------------------------------------------------------------------------- wire writing


def _enc_varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(fno: int, wt: int) -> bytes:
    return _enc_varint((fno << 3) | wt)


def _ld(fno: int, payload: bytes) -> bytes:
    return _key(fno, 2) + _enc_varint(len(payload)) + payload


def _vi(fno: int, v: int) -> bytes:
    return _key(fno, 0) + _enc_varint(v)


def encode_tensor(name: str, arr: np.ndarray, use_raw: bool = True) -> bytes:
    arr = np.ascontiguousarray(arr)
    out = b"".join(_vi(1, int(d)) for d in arr.shape)
    if arr.dtype == np.int64:
        out += _vi(2, 7)
        if use_raw:
            out += _ld(9, arr.astype("<i8").tobytes())
        else:
            out += _ld(7, b"".join(_enc_varint(int(x)) for x in arr.ravel()))
    else:
        out += _vi(2, 1)
        if use_raw:
            out += _ld(9, arr.astype("<f4").tobytes())
        else:
            out += _ld(4, arr.astype("<f4").tobytes())
    out += _ld(8, name.encode())
    return out


def encode_attr_ints(name: str, ints) -> bytes:
    return _ld(1, name.encode()) + _vi(20, 7) + b"".join(_vi(8, int(i)) for i in ints)


def encode_attr_int(name: str, i: int) -> bytes:
    return _ld(1, name.encode()) + _vi(20, 2) + _vi(3, int(i))


def encode_attr_float(name: str, f: float) -> bytes:
    return _ld(1, name.encode()) + _vi(20, 1) + _key(2, 5) + struct.pack("<f", f)


def encode_attr_string(name: str, s: str) -> bytes:
    return _ld(1, name.encode()) + _vi(20, 3) + _ld(4, s.encode())


def encode_node(op_type: str, inputs, outputs, name: str = "", attrs=()) -> bytes:
    out = b"".join(_ld(1, i.encode()) for i in inputs)
    out += b"".join(_ld(2, o.encode()) for o in outputs)
    if name:
        out += _ld(3, name.encode())
    out += _ld(4, op_type.encode())
    out += b"".join(_ld(5, a) for a in attrs)
    return out


def encode_value_info(name: str, shape, elem_type: int = 1) -> bytes:
    dims = b"".join(_ld(1, _vi(1, int(d))) for d in shape)
    tensor_type = _vi(1, elem_type) + _ld(2, dims)
    return _ld(1, name.encode()) + _ld(2, _ld(1, tensor_type))


def encode_model(graph_name: str, nodes, initializers, inputs, outputs, opset: int = 8,
                 producer: str = "ore-synth") -> bytes:
    g = b"".join(_ld(1, n) for n in nodes)
    g += _ld(2, graph_name.encode())
    g += b"".join(_ld(5, t) for t in initializers)
    g += b"".join(_ld(11, v) for v in inputs)
    g += b"".join(_ld(12, v) for v in outputs)
    m = _vi(1, 3) + _ld(2, producer.encode()) + _ld(7, g)
    m += _ld(8, _ld(1, b"") + _vi(2, opset))
    return m
