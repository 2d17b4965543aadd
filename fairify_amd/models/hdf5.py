"""Minimal, dependency-free HDF5 reader for Keras weight files.

``h5py`` is not available in the framework's Python, and the reference loads its model zoo
(``models/*/*.h5``, C02) through ``keras.models.load_model`` (``src/AC/Verify-AC.py:92-99``).
This reader implements exactly the subset of the HDF5 file format that Keras 2.x writes with
h5py's default ``libver='earliest'``: superblock v0/v1, version-1 object headers with
continuation blocks, symbol-table groups (v1 B-trees + local heaps + SNOD nodes), dataspace /
datatype / data-layout (compact + contiguous) messages, and attributes with fixed-length or
variable-length (global-heap) strings.  It executes nothing from the file (no pickle), so it is
safe on untrusted checkpoints.  Unsupported features raise ``HDF5Error``.
"""
from __future__ import annotations

import struct
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class HDF5Error(RuntimeError):
    pass


class _Datatype:
    def __init__(self, cls: int, size: int, bitfield: int, props: bytes, base: Optional["_Datatype"] = None):
        self.cls = cls
        self.size = size
        self.bitfield = bitfield
        self.props = props
        self.base = base

    @property
    def is_vlen_string(self) -> bool:
        return self.cls == 9 and (self.bitfield & 0xF) == 1

    def numpy_dtype(self) -> np.dtype:
        little = (self.bitfield & 1) == 0
        order = "<" if little else ">"
        if self.cls == 1:  # floating point
            return np.dtype(f"{order}f{self.size}")
        if self.cls == 0:  # fixed-point
            signed = bool(self.bitfield & 0x8)
            return np.dtype(f"{order}{'i' if signed else 'u'}{self.size}")
        if self.cls == 3:  # fixed-length string
            return np.dtype(f"S{self.size}")
        raise HDF5Error(f"unsupported datatype class {self.cls}")


class _Object:
    def __init__(self):
        self.messages: List[Tuple[int, bytes]] = []

    def find(self, mtype: int) -> List[bytes]:
        return [d for t, d in self.messages if t == mtype]


class H5File:
    """Read-only view of an HDF5 file: ``f['a/b']`` -> group dict / numpy array; ``attrs(path)``."""

    def __init__(self, path: str):
        with open(path, "rb") as fh:
            self.buf = fh.read()
        base = self.buf.find(SIGNATURE)
        if base < 0 or base % 512:
            raise HDF5Error("not an HDF5 file")
        self.base = base
        b = self.buf
        ver = b[base + 8]
        if ver not in (0, 1):
            raise HDF5Error(f"superblock version {ver} not supported")
        self.so = b[base + 13]
        self.sl = b[base + 14]
        if self.so != 8 or self.sl != 8:
            raise HDF5Error("only 8-byte offsets/lengths supported")
        p = base + 16 + 4 + 4  # sig+versions(8) ; leafK, internalK (4) ; flags (4)
        if ver == 1:
            p += 4
        p += 4 * 8  # base addr, free-space, eof, driver
        # root group symbol table entry
        self.root_addr = self._u64(p + 8)
        self._gheap_cache: Dict[int, Dict[int, bytes]] = {}

    # ------------------------------------------------------------------ primitive readers
    def _u8(self, p):
        return self.buf[p]

    def _u16(self, p):
        return struct.unpack_from("<H", self.buf, p)[0]

    def _u32(self, p):
        return struct.unpack_from("<I", self.buf, p)[0]

    def _u64(self, p):
        return struct.unpack_from("<Q", self.buf, p)[0]

    def _addr(self, a):
        return self.base + a

    # ------------------------------------------------------------------ object headers
    def _object(self, addr: int) -> _Object:
        p = self._addr(addr)
        version = self._u8(p)
        if version != 1:
            raise HDF5Error(f"object header version {version} not supported")
        nmsg = self._u16(p + 2)
        hsize = self._u32(p + 8)
        obj = _Object()
        blocks = [(p + 16, hsize)]
        while blocks and len(obj.messages) < nmsg:
            start, size = blocks.pop(0)
            q, end = start, start + size
            while q + 8 <= end and len(obj.messages) < nmsg:
                mtype = self._u16(q)
                msize = self._u16(q + 2)
                data = self.buf[q + 8:q + 8 + msize]
                q += 8 + msize
                if mtype == 0x10:  # continuation
                    blocks.append((self._addr(struct.unpack_from("<Q", data, 0)[0]),
                                   struct.unpack_from("<Q", data, 8)[0]))
                obj.messages.append((mtype, data))
        return obj

    # ------------------------------------------------------------------ messages
    @staticmethod
    def _dataspace(d: bytes) -> Tuple[int, ...]:
        version, rank, flags = d[0], d[1], d[2]
        off = 8 if version == 1 else 4
        if version == 2 and d[3] == 2:  # null dataspace
            return ()
        dims = struct.unpack_from("<" + "Q" * rank, d, off)
        return tuple(int(x) for x in dims)

    def _datatype(self, d: bytes, off: int = 0) -> Tuple[_Datatype, int]:
        cv = d[off]
        cls, version = cv & 0x0F, cv >> 4
        bitfield = d[off + 1] | (d[off + 2] << 8) | (d[off + 3] << 16)
        size = struct.unpack_from("<I", d, off + 4)[0]
        p = off + 8
        if cls == 9:  # variable length: base type follows
            base, used = self._datatype(d, p)
            return _Datatype(cls, size, bitfield, b"", base), (p + used) - off
        if cls == 1:
            props = d[p:p + 12]
            return _Datatype(cls, size, bitfield, props), 8 + 12
        if cls == 0:
            return _Datatype(cls, size, bitfield, d[p:p + 4]), 8 + 4
        if cls == 3:
            return _Datatype(cls, size, bitfield, b""), 8
        raise HDF5Error(f"unsupported datatype class {cls}")

    def _layout(self, d: bytes) -> Tuple[str, Any]:
        version = d[0]
        if version == 3:
            cls = d[1]
            if cls == 0:
                sz = struct.unpack_from("<H", d, 2)[0]
                return "compact", d[4:4 + sz]
            if cls == 1:
                addr, size = struct.unpack_from("<QQ", d, 2)
                return "contiguous", (addr, size)
            raise HDF5Error("chunked storage not supported")
        if version in (1, 2):
            rank, cls = d[1], d[2]
            p = 8
            if cls in (1, 2):
                addr = struct.unpack_from("<Q", d, p)[0]
                p += 8
            else:
                addr = None
            p += 4 * rank
            if cls == 0:
                sz = struct.unpack_from("<I", d, p)[0]
                return "compact", d[p + 4:p + 4 + sz]
            if cls == 1:
                return "contiguous", (addr, None)
            raise HDF5Error("chunked storage not supported")
        raise HDF5Error(f"layout version {version} not supported")

    def _gheap_object(self, coll_addr: int, index: int) -> bytes:
        if coll_addr not in self._gheap_cache:
            p = self._addr(coll_addr)
            if self.buf[p:p + 4] != b"GCOL":
                raise HDF5Error("bad global heap")
            csize = self._u64(p + 8)
            q, end = p + 16, p + csize
            objs = {}
            while q + 16 <= end:
                idx = self._u16(q)
                osize = self._u64(q + 8)
                if idx == 0:
                    break
                objs[idx] = self.buf[q + 16:q + 16 + osize]
                q += 16 + ((osize + 7) & ~7)
            self._gheap_cache[coll_addr] = objs
        return self._gheap_cache[coll_addr][index]

    def _decode(self, dt: _Datatype, shape: Tuple[int, ...], raw: bytes):
        n = int(np.prod(shape)) if shape else 1
        if dt.is_vlen_string:
            out = []
            for i in range(n):
                ln, coll, idx = struct.unpack_from("<IQI", raw, i * 16)
                s = self._gheap_object(coll, idx)[:ln] if ln else b""
                out.append(s.decode("utf-8", errors="replace"))
            return out[0] if not shape else np.array(out, dtype=object).reshape(shape)
        npdt = dt.numpy_dtype()
        arr = np.frombuffer(raw, dtype=npdt, count=n).copy()
        if dt.cls == 3:
            vals = [v.rstrip(b"\x00").decode("utf-8", errors="replace") for v in arr]
            return vals[0] if not shape else np.array(vals, dtype=object).reshape(shape)
        return arr.reshape(shape) if shape else arr[0]

    def _attrs(self, obj: _Object) -> Dict[str, Any]:
        out = {}
        for d in obj.find(0x0C):
            version = d[0]
            if version == 1:
                nsz, tsz, ssz = struct.unpack_from("<HHH", d, 2)
                p = 8
                pad = lambda x: (x + 7) & ~7
                name = d[p:p + nsz].rstrip(b"\x00").decode()
                p += pad(nsz)
                dt, _ = self._datatype(d, p)
                p += pad(tsz)
                shape = self._dataspace(d[p:p + ssz])
                p += pad(ssz)
            elif version in (2, 3):
                nsz, tsz, ssz = struct.unpack_from("<HHH", d, 2)
                p = 8 if version == 2 else 9
                name = d[p:p + nsz].rstrip(b"\x00").decode()
                p += nsz
                dt, _ = self._datatype(d, p)
                p += tsz
                shape = self._dataspace(d[p:p + ssz])
                p += ssz
            else:
                raise HDF5Error(f"attribute version {version} not supported")
            out[name] = self._decode(dt, shape, d[p:])
        return out

    # ------------------------------------------------------------------ groups
    def _heap_name(self, heap_addr: int, off: int) -> str:
        p = self._addr(heap_addr)
        if self.buf[p:p + 4] != b"HEAP":
            raise HDF5Error("bad local heap")
        data = self._addr(self._u64(p + 24))
        end = self.buf.index(b"\x00", data + off)
        return self.buf[data + off:end].decode()

    def _btree_children(self, btree_addr: int, heap_addr: int) -> Dict[str, int]:
        out: Dict[str, int] = {}
        p = self._addr(btree_addr)
        if self.buf[p:p + 4] != b"TREE":
            raise HDF5Error("bad B-tree node")
        level = self._u8(p + 5)
        used = self._u16(p + 6)
        q = p + 24
        children = []
        for i in range(used):
            q += 8  # key
            children.append(self._u64(q))
            q += 8
        for c in children:
            if level > 0:
                out.update(self._btree_children(c, heap_addr))
                continue
            s = self._addr(c)
            if self.buf[s:s + 4] != b"SNOD":
                raise HDF5Error("bad symbol table node")
            nsym = self._u16(s + 6)
            e = s + 8
            for k in range(nsym):
                name_off = self._u64(e)
                oh = self._u64(e + 8)
                out[self._heap_name(heap_addr, name_off)] = oh
                e += 40
        return out

    def _resolve(self, path: str) -> int:
        addr = self.root_addr
        for part in [p for p in path.strip("/").split("/") if p]:
            kids = self._group_members(addr)
            if part not in kids:
                raise KeyError(path)
            addr = kids[part]
        return addr

    def _group_members(self, addr: int) -> Dict[str, int]:
        obj = self._object(addr)
        st = obj.find(0x11)
        if not st:
            raise HDF5Error("object is not a (symbol-table) group")
        btree, heap = struct.unpack_from("<QQ", st[0], 0)
        return self._btree_children(btree, heap)

    # ------------------------------------------------------------------ public API
    def keys(self, path: str = "/") -> List[str]:
        return list(self._group_members(self._resolve(path)).keys())

    def is_dataset(self, path: str) -> bool:
        return bool(self._object(self._resolve(path)).find(0x08))

    def attrs(self, path: str = "/") -> Dict[str, Any]:
        return self._attrs(self._object(self._resolve(path)))

    def dataset(self, path: str) -> np.ndarray:
        obj = self._object(self._resolve(path))
        shape = self._dataspace(obj.find(0x01)[0])
        dt, _ = self._datatype(obj.find(0x03)[0])
        kind, info = self._layout(obj.find(0x08)[0])
        n = int(np.prod(shape)) if shape else 1
        if kind == "compact":
            raw = info
        else:
            addr, _ = info
            if addr == UNDEF:
                return np.zeros(shape, dtype=dt.numpy_dtype())
            start = self._addr(addr)
            raw = self.buf[start:start + n * dt.size]
        return self._decode(dt, shape, raw)

    def __getitem__(self, path: str):
        return self.dataset(path) if self.is_dataset(path) else self.keys(path)
