"""Wire protocol for the TCP data/control plane.

The reference pickles every message with ``torch.save`` into ``results/*.pt`` on disk, reads
the bytes back and ships them as one ZMQ frame; the receiver writes them to disk again and
``torch.load``s them (``/root/reference/utils/node_worker.py:44-67``).
That is a disk round trip per hop, a race between processes sharing a CWD, and arbitrary
code execution on receipt (unpickling).

Here a message is encoded in memory as::

    b"LSAM" | u32 header_len | header (UTF-8 JSON) | pad to 8 | tensor buffers (8-aligned)

The JSON header holds the object tree with tensors replaced by ``{"__t__": i}`` references
into a tensor table (dtype, shape, byte offset, length). Decoding creates tensors directly
from the received buffer (CPU); nothing is ever unpickled. Supported values: dict (str keys),
list, tuple, str, int, float, bool, None, torch.Tensor (any dtype, including bfloat16).

Message kinds used by the runtime mirror the reference's:
``input_token_info`` {hidden_states, batch_size, seq_len}, ``next_state_info`` {hidden_states,
cos, sin}, a bare next-token Tensor, the clear-KV command, profiler commands, configs.
"""
from __future__ import annotations

import json
import struct
from typing import Any

import numpy as np
import torch

MAGIC = b"LSAM"

_DT = {
    torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16", torch.float64: "f64",
    torch.int64: "i64", torch.int32: "i32", torch.int16: "i16", torch.int8: "i8", torch.uint8: "u8",
    torch.bool: "bool",
}
_TD = {v: k for k, v in _DT.items()}
# numpy carrier dtype for the raw bytes (bf16 travels as int16 bits)
_NP = {"f32": np.float32, "f16": np.float16, "bf16": np.int16, "f64": np.float64, "i64": np.int64,
       "i32": np.int32, "i16": np.int16, "i8": np.int8, "u8": np.uint8, "bool": np.bool_}


def _raw_bytes(t: torch.Tensor) -> bytes:
    t = t.detach()
    if t.device.type != "cpu":
        t = t.cpu()
    t = t.contiguous()
    if t.dtype == torch.bfloat16:
        t = t.view(torch.int16)
    return t.numpy().tobytes()


def encode(obj: Any) -> bytes:
    tensors: list = []

    def walk(o):
        if isinstance(o, torch.Tensor):
            tensors.append(o)
            return {"__t__": len(tensors) - 1}
        if isinstance(o, dict):
            for k in o:
                if not isinstance(k, str):
                    raise TypeError(f"protocol: dict keys must be str, got {type(k)}")
            return {"__d__": {k: walk(v) for k, v in o.items()}}
        if isinstance(o, tuple):
            return {"__tuple__": [walk(v) for v in o]}
        if isinstance(o, list):
            return [walk(v) for v in o]
        if o is None or isinstance(o, (bool, int, float, str)):
            return o
        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
        raise TypeError(f"protocol: cannot encode {type(o)}")

    tree = walk(obj)
    table, blobs, off = [], [], 0
    for t in tensors:
        b = _raw_bytes(t)
        table.append({"dt": _DT[t.dtype], "shape": list(t.shape), "off": off, "n": len(b)})
        pad = (-len(b)) % 8
        blobs.append(b + b"\0" * pad)
        off += len(b) + pad
    hdr = json.dumps({"v": 1, "obj": tree, "t": table}, separators=(",", ":")).encode()
    hpad = (-(8 + len(hdr))) % 8
    return b"".join([MAGIC, struct.pack("<I", len(hdr)), hdr, b"\0" * hpad] + blobs)


def decode(data: bytes) -> Any:
    if len(data) < 8 or data[:4] != MAGIC:
        raise ValueError("protocol: bad magic (not an LSAM message)")
    (hl,) = struct.unpack("<I", data[4:8])
    hdr = json.loads(data[8:8 + hl].decode())
    base = 8 + hl + ((-(8 + hl)) % 8)
    mv = memoryview(data)
    tens = []
    for e in hdr["t"]:
        dt = e["dt"]
        arr = np.frombuffer(mv[base + e["off"]: base + e["off"] + e["n"]], dtype=_NP[dt]).reshape(e["shape"])
        t = torch.from_numpy(arr.copy())
        if dt == "bf16":
            t = t.view(torch.bfloat16)
        tens.append(t)

    def walk(o):
        if isinstance(o, dict):
            if "__t__" in o:
                return tens[o["__t__"]]
            if "__d__" in o:
                return {k: walk(v) for k, v in o["__d__"].items()}
            if "__tuple__" in o:
                return tuple(walk(v) for v in o["__tuple__"])
            raise ValueError("protocol: malformed header")
        if isinstance(o, list):
            return [walk(v) for v in o]
        return o

    return walk(hdr["obj"])


def is_json_message(data: bytes) -> bool:
    return not data.startswith(MAGIC)
