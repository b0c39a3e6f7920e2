"""Point-registry snapshots: read (and write) the reference's ``state.pkl`` without unpickling.

Reference: ``Point.snapshot`` / ``Point.backup`` (gym/engine.py:199-212, gym/optimized_engine.py:319-336)
pickle ``{"points": [gym.engine.Point, ...], "r_points": {...}}`` with protocol 4.  Each ``Point``
carries ``m`` (Python float), ``pos``/``v``/``a``/``old_a`` (float32 ndarrays rebuilt through
``numpy._core.multiarray._reconstruct``; ``old_a`` is memo-aliased to ``a``), ``r``, ``color``, ``e``.

Loading that file with ``pickle`` would execute the globals it names.  This module never does: it
walks the opcode stream with :func:`pickletools.genops` (a disassembler, executes nothing) and runs
a tiny *data-only* stack machine that understands the opcodes such a snapshot uses.  Every global the
stream names is kept as an inert ``_Global(module, name)`` tag; only the two numpy reconstructors and
``gym.engine.Point`` (and its G2 twin) are recognised, and they are interpreted as plain data.

:func:`write_snapshot` emits the same protocol-4 shape from batched arrays so the reference's
``Point.backup`` (a pickle load on THEIR side) can read states produced here.
"""
from __future__ import annotations

import io
import pickletools
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List

import numpy as np

__all__ = ["SnapshotPoint", "read_snapshot", "read_snapshot_bytes", "write_snapshot", "SnapshotError"]


class SnapshotError(ValueError):
    pass


@dataclass
class SnapshotPoint:
    m: float
    pos: np.ndarray
    v: np.ndarray
    a: np.ndarray
    old_a: np.ndarray
    r: float = 1.0
    color: Any = "black"
    e: float = 1.6e-19
    extra: Dict[str, Any] = field(default_factory=dict)


class _Global:
    __slots__ = ("module", "name")

    def __init__(self, module: str, name: str):
        self.module, self.name = module, name

    def __repr__(self):
        return f"<global {self.module}.{self.name}>"


class _Obj:
    """An object built by NEWOBJ/REDUCE, kept as data (class tag + args + state)."""
    __slots__ = ("cls", "args", "state")

    def __init__(self, cls, args):
        self.cls, self.args, self.state = cls, args, None


_MARK = object()
_POINT_CLASSES = {("gym.engine", "Point"), ("engine", "Point"), ("optimized_engine", "Point"),
                  ("gym.optimized_engine", "Point"), ("gym.engine", "DingPoint"),
                  ("optimized_engine", "DingPoint")}
_RECONSTRUCT = {("numpy._core.multiarray", "_reconstruct"), ("numpy.core.multiarray", "_reconstruct")}
_NDARRAY = {("numpy", "ndarray")}
_DTYPE = {("numpy", "dtype")}


def _ndarray_from(obj: _Obj) -> np.ndarray:
    # state = (version, shape, dtype_obj, is_fortran, raw_bytes)
    st = obj.state
    if not (isinstance(st, tuple) and len(st) == 5):
        raise SnapshotError("unexpected ndarray state")
    _, shape, dt, fortran, raw = st
    if not (isinstance(dt, _Obj) and isinstance(dt.cls, _Global)
            and (dt.cls.module, dt.cls.name) in _DTYPE):
        raise SnapshotError("unexpected dtype record")
    code = dt.args[0]
    if code not in ("f4", "f8", "i4", "i8"):
        raise SnapshotError(f"unsupported dtype {code!r}")
    order = ">" if isinstance(dt.state, tuple) and dt.state[1] == ">" else "<"
    arr = np.frombuffer(bytes(raw), dtype=np.dtype(order + code)).copy()
    return arr.reshape(shape, order="F" if fortran else "C")


def _materialise(x):
    if isinstance(x, _Obj) and isinstance(x.cls, _Global):
        key = (x.cls.module, x.cls.name)
        if key in _RECONSTRUCT:
            return _ndarray_from(x)
    return x


def read_snapshot_bytes(data: bytes):
    """Parse snapshot bytes into ``(points: list[SnapshotPoint], r_points: dict)``. Executes nothing."""
    stack: List[Any] = []
    memo: Dict[int, Any] = {}
    arrays_by_id: Dict[int, np.ndarray] = {}

    def pop_mark():
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        items.reverse()
        return items

    result = None
    for op, arg, _pos in pickletools.genops(io.BytesIO(data)):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        elif name == "MARK":
            stack.append(_MARK)
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif name in ("BINPUT", "LONG_BINPUT"):
            memo[arg] = stack[-1]
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE"):
            stack.append(str(arg))
        elif name in ("SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(bytes(arg))
        elif name in ("BININT1", "BININT2", "BININT", "LONG1", "INT"):
            stack.append(int(arg))
        elif name in ("BINFLOAT", "FLOAT"):
            stack.append(float(arg))
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "NONE":
            stack.append(None)
        elif name == "TUPLE1":
            stack.append((stack.pop(),))
        elif name == "TUPLE2":
            b = stack.pop(); a = stack.pop(); stack.append((a, b))
        elif name == "TUPLE3":
            c = stack.pop(); b = stack.pop(); a = stack.pop(); stack.append((a, b, c))
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "STACK_GLOBAL":
            nm = stack.pop(); mod = stack.pop()
            stack.append(_Global(mod, nm))
        elif name == "GLOBAL":
            mod, nm = arg.split(" ", 1)
            stack.append(_Global(mod, nm))
        elif name in ("REDUCE", "NEWOBJ"):
            args = stack.pop(); cls = stack.pop()
            stack.append(_Obj(cls, args))
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, _Obj):
                raise SnapshotError("BUILD on non-object")
            obj.state = state
        elif name == "SETITEMS":
            items = pop_mark(); d = stack[-1]
            for k in range(0, len(items), 2):
                d[items[k]] = items[k + 1]
        elif name == "SETITEM":
            v = stack.pop(); k = stack.pop(); stack[-1][k] = v
        elif name == "APPENDS":
            items = pop_mark(); stack[-1].extend(items)
        elif name == "APPEND":
            v = stack.pop(); stack[-1].append(v)
        elif name == "STOP":
            result = stack.pop()
            break
        else:
            raise SnapshotError(f"opcode {name} not allowed in a Point snapshot")
    if not isinstance(result, dict) or "points" not in result:
        raise SnapshotError("not a Point snapshot (missing 'points')")

    points: List[SnapshotPoint] = []
    for obj in result["points"]:
        if not (isinstance(obj, _Obj) and isinstance(obj.cls, _Global)
                and (obj.cls.module, obj.cls.name) in _POINT_CLASSES):
            raise SnapshotError(f"unexpected point record {obj!r}")
        st = dict(obj.state or {})
        arrs = {}
        for key in ("pos", "v", "a", "old_a"):
            raw = st.get(key)
            if raw is None:
                continue
            if id(raw) not in arrays_by_id:
                arrays_by_id[id(raw)] = _materialise(raw)
            arrs[key] = arrays_by_id[id(raw)]
        pos = np.asarray(arrs["pos"], dtype=np.float32)
        v = np.asarray(arrs.get("v", np.zeros(3, np.float32)), dtype=np.float32)
        a = np.asarray(arrs.get("a", np.zeros_like(v)), dtype=np.float32)
        old_a = np.asarray(arrs.get("old_a", a), dtype=np.float32)
        extra = {k: st[k] for k in st if k not in ("m", "pos", "v", "a", "old_a", "r", "color", "e")}
        points.append(SnapshotPoint(m=float(st["m"]), pos=pos.copy(), v=v.copy(), a=a.copy(),
                                    old_a=old_a.copy(), r=float(st.get("r", 1.0)),
                                    color=st.get("color", "black"), e=float(st.get("e", 1.6e-19)),
                                    extra=extra))
    r_points = result.get("r_points", {})
    if r_points:
        # keys are tuples of Point records; keep only what is data (rest lengths by point index)
        idx = {id(o): k for k, o in enumerate(result["points"])}
        conv = {}
        for key, val in r_points.items():
            conv[tuple(idx.get(id(o), -1) for o in key)] = float(val) if not isinstance(val, _Obj) else val
        r_points = conv
    return points, r_points


def read_snapshot(path: str):
    with open(path, "rb") as f:
        return read_snapshot_bytes(f.read())


# --------------------------------------------------------------------------------------------- writer
class _W:
    """Minimal protocol-4 opcode emitter (memoises strings like the stdlib pickler does)."""

    def __init__(self):
        self.b = io.BytesIO()
        self.memo = 0
        self.strs: Dict[str, int] = {}

    def op(self, code: bytes, payload: bytes = b""):
        self.b.write(code + payload)

    def memoize(self) -> int:
        self.op(b"\x94"); i = self.memo; self.memo += 1; return i

    def get(self, i: int):
        if i < 256:
            self.op(b"h", bytes([i]))
        else:
            self.op(b"j", struct.pack("<I", i))

    def s(self, text: str):
        if text in self.strs:
            self.get(self.strs[text]); return
        e = text.encode("utf-8")
        if len(e) < 256:
            self.op(b"\x8c", bytes([len(e)]) + e)
        else:
            self.op(b"X", struct.pack("<I", len(e)) + e)
        self.strs[text] = self.memoize()

    def bfloat(self, x: float):
        self.op(b"G", struct.pack(">d", float(x)))

    def sbytes(self, raw: bytes) -> int:
        if len(raw) < 256:
            self.op(b"C", bytes([len(raw)]) + raw)
        else:
            self.op(b"B", struct.pack("<I", len(raw)) + raw)
        return self.memoize()


def write_snapshot(path: str, m, pos, v, a=None, old_a=None, r=None, color="black", e=1.6e-19) -> None:
    """Write a protocol-4 ``state.pkl`` with the same opcode shape as ``Point.snapshot``.

    ``m [P]``, ``pos/v/a/old_a [P,3]`` float32.  ``old_a`` defaults to aliasing ``a`` as
    gym/engine.py:49 does.  Points are tagged ``gym.engine.Point``; ``r_points`` is left empty.
    """
    m = np.asarray(m, dtype=np.float64).reshape(-1)
    pos = np.ascontiguousarray(pos, dtype=np.float32).reshape(-1, 3)
    v = np.ascontiguousarray(v, dtype=np.float32).reshape(-1, 3)
    a = np.zeros_like(v) if a is None else np.ascontiguousarray(a, dtype=np.float32).reshape(-1, 3)
    alias_old = old_a is None
    old_a = a if alias_old else np.ascontiguousarray(old_a, dtype=np.float32).reshape(-1, 3)
    P = len(m)
    r = np.broadcast_to(np.asarray(m ** 0.3 if r is None else r, dtype=np.float64), (P,))
    w = _W()
    memo: Dict[str, int] = {}

    def arr(x: np.ndarray) -> int:
        if "recon" not in memo:
            w.s("numpy._core.multiarray"); w.s("_reconstruct"); w.op(b"\x93"); memo["recon"] = w.memoize()
            w.s("numpy"); w.s("ndarray"); w.op(b"\x93"); memo["nd"] = w.memoize()
        else:
            w.get(memo["recon"]); w.get(memo["nd"])
        w.op(b"K", b"\x00"); w.op(b"\x85"); w.memoize()
        if "b" not in memo:
            memo["b"] = w.sbytes(b"b")
        else:
            w.get(memo["b"])
        w.op(b"\x87"); w.memoize(); w.op(b"R"); obj = w.memoize()
        w.op(b"("); w.op(b"K", b"\x01"); w.op(b"K", b"\x03"); w.op(b"\x85"); w.memoize()
        if "dt" not in memo:
            w.s("numpy"); w.s("dtype"); w.op(b"\x93"); w.memoize()
            w.s("f4"); w.op(b"\x89"); w.op(b"\x88"); w.op(b"\x87"); w.memoize(); w.op(b"R")
            memo["dt"] = w.memoize()
            w.op(b"("); w.op(b"K", b"\x03"); w.s("<"); w.op(b"N"); w.op(b"N"); w.op(b"N")
            w.op(b"J", struct.pack("<i", -1)); w.op(b"J", struct.pack("<i", -1)); w.op(b"K", b"\x00")
            w.op(b"t"); w.memoize(); w.op(b"b")
        else:
            w.get(memo["dt"])
        w.op(b"\x89"); w.sbytes(np.ascontiguousarray(x, dtype="<f4").tobytes()); w.op(b"t")
        w.memoize(); w.op(b"b")
        return obj

    w.op(b"\x80\x04")
    w.op(b"}"); w.memoize(); w.op(b"(")
    w.s("points"); w.op(b"]"); w.memoize(); w.op(b"(")
    for p in range(P):
        if "cls" not in memo:
            w.s("gym.engine"); w.s("Point"); w.op(b"\x93"); memo["cls"] = w.memoize()
        else:
            w.get(memo["cls"])
        w.op(b")"); w.op(b"\x81"); w.memoize(); w.op(b"}"); w.memoize(); w.op(b"(")
        w.s("m"); w.bfloat(m[p])
        w.s("pos"); arr(pos[p])
        w.s("v"); arr(v[p])
        w.s("a"); a_obj = arr(a[p])
        w.s("r"); w.bfloat(r[p])
        w.s("old_a")
        if alias_old:
            w.get(a_obj)
        else:
            arr(old_a[p])
        w.s("color"); w.s(str(color))
        w.s("e"); w.bfloat(e)
        w.op(b"u"); w.op(b"b")
    w.op(b"e")
    w.s("r_points"); w.op(b"}"); w.memoize()
    w.op(b"u"); w.op(b".")
    with open(path, "wb") as f:
        f.write(w.b.getvalue())
