"""Minimal reader for USD binary "crate" files (``.usdc`` / ``.usd`` with a
``PXR-USDC`` header).

The reference drives Omniverse and reads its scene through ``pxr``
(``usd.get_context().get_stage()``, generate_construction_data.py:1370;
``stage.GetPrimAtPath`` / ``UsdGeom.Xform`` at :592-597).  ``pxr`` is not
available in this build, so this module decodes the on-disk crate format
directly — enough of it to pull mesh geometry, primvars, xform ops and
material bindings out of ``cad_models/world2.usd.backup`` (crate v0.8.0).

Format summary (public OpenUSD crate layout):

* 88-byte bootstrap: ``b"PXR-USDC"``, 8 version bytes, int64 TOC offset.
* TOC: uint64 count, then ``(char[16] name, int64 start, int64 size)``.
* Sections TOKENS / STRINGS / FIELDS / FIELDSETS / PATHS / SPECS.
* Structural sections are LZ4-block compressed ("TfFastCompression") and
  integer arrays additionally use USD's 2-bit-code delta encoding.
* Every value is a 64-bit ``ValueRep``: bit63 array, bit62 inlined,
  bit61 compressed, bits48-55 type enum, bits0-47 payload/offset.

Only host-side scene IO: nothing here is on the GPU hot path.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

__all__ = ["CrateFile", "lz4_block_decompress", "fast_decompress", "decode_integers"]


# --------------------------------------------------------------------------
# Compression primitives
# --------------------------------------------------------------------------

def lz4_block_decompress(src: bytes, max_out: int) -> bytes:
    """Decode one raw LZ4 block (no frame header)."""
    out = bytearray()
    i, n = 0, len(src)
    while i < n:
        token = src[i]
        i += 1
        lit = token >> 4
        if lit == 15:
            while True:
                b = src[i]
                i += 1
                lit += b
                if b != 255:
                    break
        if lit:
            out += src[i:i + lit]
            i += lit
        if i >= n:
            break
        off = src[i] | (src[i + 1] << 8)
        i += 2
        mlen = token & 15
        if mlen == 15:
            while True:
                b = src[i]
                i += 1
                mlen += b
                if b != 255:
                    break
        mlen += 4
        start = len(out) - off
        if off >= mlen:
            out += out[start:start + mlen]
        else:  # overlapping copy: repeat the period
            chunk = out[start:]
            reps, rem = divmod(mlen, off)
            out += chunk * reps + chunk[:rem]
        if len(out) > max_out:
            raise ValueError("lz4: output overflow")
    return bytes(out)


def fast_decompress(src: bytes, max_out: int) -> bytes:
    """TfFastCompression::DecompressFromBuffer: 1 chunk-count byte, then
    either one LZ4 block (count 0) or ``count`` (int32 size, block) pairs."""
    nchunks = src[0]
    if nchunks == 0:
        return lz4_block_decompress(src[1:], max_out)
    pos, parts = 1, []
    for _ in range(nchunks):
        (sz,) = struct.unpack_from("<i", src, pos)
        pos += 4
        parts.append(lz4_block_decompress(src[pos:pos + sz], max_out))
        pos += sz
    return b"".join(parts)


def _encoded_buffer_size(n: int, width: int) -> int:
    return width + (n * 2 + 7) // 8 + n * width if n else 0


def decode_integers(buf: bytes, n: int, width: int) -> np.ndarray:
    """Usd_IntegerCompression decode (after LZ4): common value, 2-bit codes
    (0 common, 1 small, 2 medium, 3 full width), then deltas; prefix-summed."""
    if n == 0:
        return np.zeros(0, np.int64)
    sdt = {4: "<i4", 8: "<i8"}[width]
    small, med = ({4: ("<i1", "<i2"), 8: ("<i2", "<i4")})[width]
    common = int(np.frombuffer(buf, sdt, 1, 0)[0])
    ncode = (n * 2 + 7) // 8
    codes = np.frombuffer(buf, np.uint8, ncode, width)
    codes = np.stack([(codes >> (2 * k)) & 3 for k in range(4)], 1).reshape(-1)[:n]
    sizes = np.array([0, np.dtype(small).itemsize, np.dtype(med).itemsize, width])[codes]
    offs = width + ncode + np.concatenate([[0], np.cumsum(sizes)[:-1]])
    vals = np.full(n, common, np.int64)
    raw = np.frombuffer(buf, np.uint8)
    for code, dt in ((1, small), (2, med), (3, sdt)):
        sel = np.nonzero(codes == code)[0]
        if sel.size:
            isz = np.dtype(dt).itemsize
            idx = offs[sel][:, None] + np.arange(isz)[None, :]
            vals[sel] = raw[idx].copy().view(dt).reshape(-1).astype(np.int64)
    return np.cumsum(vals)


# --------------------------------------------------------------------------
# Crate types
# --------------------------------------------------------------------------

T = {  # crateDataTypes enum (subset that matters here)
    "Invalid": 0, "Bool": 1, "UChar": 2, "Int": 3, "UInt": 4, "Int64": 5, "UInt64": 6,
    "Half": 7, "Float": 8, "Double": 9, "String": 10, "Token": 11, "AssetPath": 12,
    "Matrix2d": 13, "Matrix3d": 14, "Matrix4d": 15, "Quatd": 16, "Quatf": 17, "Quath": 18,
    "Vec2d": 19, "Vec2f": 20, "Vec2h": 21, "Vec2i": 22, "Vec3d": 23, "Vec3f": 24,
    "Vec3h": 25, "Vec3i": 26, "Vec4d": 27, "Vec4f": 28, "Vec4h": 29, "Vec4i": 30,
    "Dictionary": 31, "TokenListOp": 32, "StringListOp": 33, "PathListOp": 34,
    "ReferenceListOp": 35, "IntListOp": 36, "Int64ListOp": 37, "UIntListOp": 38,
    "UInt64ListOp": 39, "PathVector": 40, "TokenVector": 41, "Specifier": 42,
    "Permission": 43, "Variability": 44, "VariantSelectionMap": 45, "TimeSamples": 46,
    "Payload": 47, "DoubleVector": 48, "LayerOffsetVector": 49, "StringVector": 50,
    "ValueBlock": 51, "Value": 52, "UnregisteredValue": 53,
}
TN = {v: k for k, v in T.items()}

_SCALAR = {  # type -> (numpy dtype, element count)
    T["Bool"]: ("u1", 1), T["UChar"]: ("u1", 1), T["Int"]: ("<i4", 1), T["UInt"]: ("<u4", 1),
    T["Int64"]: ("<i8", 1), T["UInt64"]: ("<u8", 1), T["Half"]: ("<f2", 1),
    T["Float"]: ("<f4", 1), T["Double"]: ("<f8", 1),
    T["Matrix2d"]: ("<f8", 4), T["Matrix3d"]: ("<f8", 9), T["Matrix4d"]: ("<f8", 16),
    T["Quatd"]: ("<f8", 4), T["Quatf"]: ("<f4", 4), T["Quath"]: ("<f2", 4),
    T["Vec2d"]: ("<f8", 2), T["Vec2f"]: ("<f4", 2), T["Vec2h"]: ("<f2", 2), T["Vec2i"]: ("<i4", 2),
    T["Vec3d"]: ("<f8", 3), T["Vec3f"]: ("<f4", 3), T["Vec3h"]: ("<f2", 3), T["Vec3i"]: ("<i4", 3),
    T["Vec4d"]: ("<f8", 4), T["Vec4f"]: ("<f4", 4), T["Vec4h"]: ("<f2", 4), T["Vec4i"]: ("<i4", 4),
}

SPEC_TYPES = {0: "Unknown", 1: "Attribute", 2: "Connection", 3: "Expression", 4: "Mapper",
              5: "MapperArg", 6: "Prim", 7: "PseudoRoot", 8: "Relationship",
              9: "RelationshipTarget", 10: "Variant", 11: "VariantSet"}


@dataclass
class Spec:
    path: str
    spec_type: str
    fields: Dict[str, Any] = field(default_factory=dict)


class CrateFile:
    """Decoded crate: ``specs`` maps SdfPath strings to :class:`Spec`."""

    def __init__(self, path: str):
        with open(path, "rb") as f:
            self.data = f.read()
        d = self.data
        if d[:8] != b"PXR-USDC":
            raise ValueError(f"{path}: not a USD crate file")
        self.version = tuple(d[8:11])
        (toc,) = struct.unpack_from("<q", d, 16)
        (nsec,) = struct.unpack_from("<Q", d, toc)
        self.sections = {}
        for i in range(nsec):
            o = toc + 8 + i * 32
            name = d[o:o + 16].rstrip(b"\0").decode()
            self.sections[name] = struct.unpack_from("<qq", d, o + 16)
        self._read_tokens()
        self._read_strings()
        self._read_fields()
        self._read_fieldsets()
        self._read_paths()
        self._read_specs()
        self._value_cache: Dict[int, Any] = {}

    # -- low-level ----------------------------------------------------------
    def _u64(self, pos: int) -> int:
        return struct.unpack_from("<Q", self.data, pos)[0]

    def _compressed_ints(self, pos: int, n: int, width: int = 4) -> Tuple[np.ndarray, int]:
        csize = self._u64(pos)
        pos += 8
        raw = fast_decompress(self.data[pos:pos + csize], _encoded_buffer_size(n, width))
        return decode_integers(raw, n, width), pos + csize

    # -- sections -----------------------------------------------------------
    def _read_tokens(self):
        pos, _ = self.sections["TOKENS"]
        ntok, usize, csize = struct.unpack_from("<QQQ", self.data, pos)
        raw = fast_decompress(self.data[pos + 24:pos + 24 + csize], usize)
        toks = raw.split(b"\0")[:ntok]
        self.tokens = [t.decode("utf-8", "replace") for t in toks]

    def _read_strings(self):
        pos, _ = self.sections["STRINGS"]
        n = self._u64(pos)
        self.strings = list(np.frombuffer(self.data, "<u4", n, pos + 8))

    def _read_fields(self):
        pos, _ = self.sections["FIELDS"]
        n = self._u64(pos)
        tok, pos = self._compressed_ints(pos + 8, n)
        rsize = self._u64(pos)
        reps = fast_decompress(self.data[pos + 8:pos + 8 + rsize], n * 8)
        self.fields = list(zip(tok.astype(int), np.frombuffer(reps, "<u8", n).tolist()))

    def _read_fieldsets(self):
        pos, _ = self.sections["FIELDSETS"]
        n = self._u64(pos)
        fs, _ = self._compressed_ints(pos + 8, n)
        self.fieldsets = (fs.astype(np.int64) & 0xFFFFFFFF).tolist()

    def _read_paths(self):
        pos, _ = self.sections["PATHS"]
        npaths = self._u64(pos)
        nenc = self._u64(pos + 8)
        pidx, p = self._compressed_ints(pos + 16, nenc)
        etok, p = self._compressed_ints(p, nenc)
        jumps, p = self._compressed_ints(p, nenc)
        pidx, etok, jumps = (a.astype(np.int64).tolist() for a in (pidx, etok, jumps))
        etok = [t - (1 << 32) if t >= (1 << 31) else t for t in etok]
        jumps = [j - (1 << 32) if j >= (1 << 31) else j for j in jumps]
        paths: List[Optional[str]] = [None] * npaths
        stack = [(0, None)]
        while stack:
            cur, parent = stack.pop()
            while True:
                this = cur
                cur += 1
                if parent is None:
                    parent = "/"
                    paths[pidx[this]] = "/"
                else:
                    t = etok[this]
                    name = self.tokens[abs(t)]
                    if t < 0:
                        paths[pidx[this]] = parent + "." + name
                    else:
                        paths[pidx[this]] = (parent.rstrip("/") + "/" + name) if not name.startswith("{") else parent + name
                j = jumps[this]
                has_child = j > 0 or j == -1
                has_sib = j >= 0
                if has_child:
                    if has_sib:
                        stack.append((this + j, parent))
                    parent = paths[pidx[this]]
                elif not has_sib:
                    break
        self.paths = paths

    def _read_specs(self):
        pos, _ = self.sections["SPECS"]
        n = self._u64(pos)
        pi, p = self._compressed_ints(pos + 8, n)
        fsi, p = self._compressed_ints(p, n)
        st, p = self._compressed_ints(p, n)
        self.specs: Dict[str, Spec] = {}
        self.spec_order: List[str] = []
        for a, b, c in zip(pi.tolist(), fsi.tolist(), st.tolist()):
            path = self.paths[a]
            spec = Spec(path, SPEC_TYPES.get(int(c), str(c)))
            i = int(b)
            while self.fieldsets[i] != 0xFFFFFFFF:
                tok, rep = self.fields[self.fieldsets[i]]
                spec.fields[self.tokens[tok]] = rep
                i += 1
            self.specs[path] = spec
            self.spec_order.append(path)

    # -- values -------------------------------------------------------------
    def value(self, rep: int) -> Any:
        """Decode a ValueRep. Unsupported kinds decode to ``("unsupported", type)``."""
        if rep in self._value_cache:
            return self._value_cache[rep]
        v = self._decode(rep)
        self._value_cache[rep] = v
        return v

    @staticmethod
    def rep_offset(rep: int) -> int:
        return rep & ((1 << 48) - 1)

    def _decode(self, rep: int) -> Any:
        is_array = bool(rep >> 63 & 1)
        inlined = bool(rep >> 62 & 1)
        compressed = bool(rep >> 61 & 1)
        ty = (rep >> 48) & 0xFF
        payload = rep & ((1 << 48) - 1)
        d = self.data
        if is_array:
            if inlined:
                return np.zeros(0)
            pos = payload
            n = self._u64(pos)
            pos += 8
            if ty in (T["Int"], T["UInt"], T["Int64"], T["UInt64"]):
                width = 4 if ty in (T["Int"], T["UInt"]) else 8
                dt = _SCALAR[ty][0]
                if compressed and n >= 16:
                    vals, _ = self._compressed_ints(pos, n, width)
                    return vals.astype(dt)
                return np.frombuffer(d, dt, n, pos).copy()
            if ty in (T["Half"], T["Float"], T["Double"]):
                dt = _SCALAR[ty][0]
                if compressed and n >= 16:
                    code = chr(d[pos])
                    pos += 1
                    if code == "i":
                        vals, _ = self._compressed_ints(pos, n, 4)
                        return vals.astype(dt)
                    if code == "t":
                        (lut_n,) = struct.unpack_from("<I", d, pos)
                        pos += 4
                        lut = np.frombuffer(d, dt, lut_n, pos)
                        pos += lut_n * np.dtype(dt).itemsize
                        idx, _ = self._compressed_ints(pos, n, 4)
                        return lut[idx.astype(np.int64)].copy()
                    raise ValueError(f"bad float array code {code!r}")
                return np.frombuffer(d, dt, n, pos).copy()
            if ty in _SCALAR:
                dt, k = _SCALAR[ty]
                return np.frombuffer(d, dt, n * k, pos).reshape(n, k).copy()
            if ty == T["Token"]:
                idx = np.frombuffer(d, "<u4", n, pos)
                return [self.tokens[i] for i in idx]
            if ty in (T["String"], T["AssetPath"]):
                idx = np.frombuffer(d, "<u4", n, pos)
                return [self.tokens[self.strings[i]] if ty == T["String"] else self.tokens[i] for i in idx]
            return ("unsupported-array", TN.get(ty, ty))
        if inlined:
            if ty in (T["Token"], T["AssetPath"]):
                return self.tokens[payload]
            if ty == T["String"]:
                return self.tokens[self.strings[payload]]
            if ty in (T["Bool"], T["UChar"], T["Specifier"], T["Variability"], T["Permission"]):
                return int(payload & 0xFF) if ty != T["Bool"] else bool(payload & 1)
            if ty in (T["Int"], T["UInt"]):
                v = payload & 0xFFFFFFFF
                return v - (1 << 32) if ty == T["Int"] and v >= (1 << 31) else v
            if ty in (T["Float"], T["Double"]):
                return struct.unpack("<f", struct.pack("<I", payload & 0xFFFFFFFF))[0]
            if ty == T["Half"]:
                return float(np.frombuffer(struct.pack("<H", payload & 0xFFFF), "<f2")[0])
            if ty in _SCALAR and ty not in (T["Matrix2d"], T["Matrix3d"], T["Matrix4d"]):
                _, k = _SCALAR[ty]
                b = struct.pack("<Q", payload)[:k]
                return np.frombuffer(b, "i1", k).astype(np.float64)
            if ty in (T["Matrix2d"], T["Matrix3d"], T["Matrix4d"]):
                k = {T["Matrix2d"]: 2, T["Matrix3d"]: 3, T["Matrix4d"]: 4}[ty]
                diag = np.frombuffer(struct.pack("<Q", payload)[:k], "i1", k).astype(np.float64)
                return np.diag(diag)
            if ty == T["ValueBlock"]:
                return None
            return ("unsupported-inline", TN.get(ty, ty))
        pos = payload
        if ty in _SCALAR:
            dt, k = _SCALAR[ty]
            v = np.frombuffer(d, dt, k, pos).astype(np.float64 if dt[-2] == "f" else np.int64)
            if ty in (T["Matrix2d"], T["Matrix3d"], T["Matrix4d"]):
                m = int(round(k ** 0.5))
                return v.reshape(m, m)
            return v if k > 1 else v[0]
        if ty == T["TokenVector"]:
            n = self._u64(pos)
            return [self.tokens[i] for i in np.frombuffer(d, "<u4", n, pos + 8)]
        if ty == T["PathListOp"] or ty == T["TokenListOp"]:
            return self._list_op(pos, ty)
        if ty == T["PathVector"]:
            n = self._u64(pos)
            return [self.paths[i] for i in np.frombuffer(d, "<u4", n, pos + 8)]
        return ("unsupported", TN.get(ty, ty))

    def _list_op(self, pos: int, ty: int) -> Dict[str, list]:
        h = self.data[pos]
        pos += 1
        out: Dict[str, list] = {"explicit": bool(h & 1)}
        for bit, key in ((2, "explicitItems"), (4, "addedItems"), (32, "prependedItems"),
                         (64, "appendedItems"), (8, "deletedItems"), (16, "orderedItems")):
            if h & bit:
                n = self._u64(pos)
                idx = np.frombuffer(self.data, "<u4", n, pos + 8)
                pos += 8 + 4 * n
                out[key] = [self.paths[i] if ty == T["PathListOp"] else self.tokens[i] for i in idx]
        return out

    # -- convenience --------------------------------------------------------
    def field(self, path: str, name: str, default: Any = None) -> Any:
        s = self.specs.get(path)
        if s is None or name not in s.fields:
            return default
        return self.value(s.fields[name])

    def rep(self, path: str, name: str) -> Optional[int]:
        s = self.specs.get(path)
        return None if s is None else s.fields.get(name)

    def children(self, path: str) -> List[str]:
        kids = self.field(path, "primChildren", []) or []
        base = path.rstrip("/")
        return [base + "/" + k for k in kids]

    def prim_type(self, path: str) -> Optional[str]:
        return self.field(path, "typeName")

    def attr(self, prim: str, name: str, default: Any = None) -> Any:
        return self.field(prim + "." + name, "default", default)
