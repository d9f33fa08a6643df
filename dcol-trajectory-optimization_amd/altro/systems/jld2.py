"""Minimal reader for the numeric datasets of a JLD2 file.

The quadrotor scene loads its polytope obstacles from systems/polytopes.jld2 through h5py
(cluttered_hallway_quadrotor.py:271-279); neither h5py nor an HDF5 library is available
here.  JLD2 files are HDF5 files behind a 512-byte user block, so this reads exactly the
HDF5 structures such a file uses for plain Float64 arrays:

  superblock v2/v3  -> root group object header (v2, "OHDR", with continuation blocks)
  link messages     -> dataset name -> dataset object header address
  dataspace msg     -> dims (C order: h5py's shape; Julia's column-major array transposed)
  datatype msg      -> IEEE float, 8 bytes, little endian (anything else is rejected)
  layout msg v3/v4  -> compact (data inline) or contiguous (address + size)

It returns what h5py's ``f[name][:]`` would, as float64 arrays.  Anything outside that
subset raises ValueError.
"""
from __future__ import annotations

import struct

import numpy as np

_SIG = b"\x89HDF\r\n\x1a\n"
_UNDEF = 0xFFFFFFFFFFFFFFFF


class _File:
    def __init__(self, raw: bytes):
        self.raw = raw
        self.base = self._find_superblock()

    def _find_superblock(self):
        off = 0
        while off < len(self.raw):
            if self.raw[off:off + 8] == _SIG:
                ver = self.raw[off + 8]
                if ver not in (2, 3):
                    raise ValueError(f"HDF5 superblock version {ver} not supported")
                so, sl = self.raw[off + 9], self.raw[off + 10]
                if so != 8 or sl != 8:
                    raise ValueError("only 8-byte offsets/lengths are supported")
                base, _ext, _eof, root = struct.unpack_from("<4Q", self.raw, off + 12)
                self.root = root
                return base
            off = 512 if off == 0 else off * 2
        raise ValueError("no HDF5 superblock found")

    def u(self, fmt, off):
        return struct.unpack_from("<" + fmt, self.raw, off)

    def messages(self, addr):
        """Yield (type, body_offset, size) of a v2 object header, following continuations."""
        p = self.base + addr
        if self.raw[p:p + 4] != b"OHDR" or self.raw[p + 4] != 2:
            raise ValueError(f"object header at {addr:#x} is not a v2 OHDR")
        flags = self.raw[p + 5]
        q = p + 6
        if flags & 0x20:
            q += 16                               # access/modification/change/birth times
        if flags & 0x10:
            q += 4                                # max compact / min dense attribute counts
        w = 1 << (flags & 3)
        size = int.from_bytes(self.raw[q:q + w], "little")
        q += w
        blocks = [(q, q + size)]
        while blocks:
            s, e = blocks.pop(0)
            while s + 4 <= e:
                mtype = self.raw[s]
                msize = self.u("H", s + 1)[0]
                s += 4 + (2 if flags & 0x04 else 0)
                if mtype == 0x10:                 # continuation -> "OCHK" block
                    caddr, clen = self.u("QQ", s)
                    c = self.base + caddr
                    if self.raw[c:c + 4] != b"OCHK":
                        raise ValueError("bad continuation block")
                    blocks.append((c + 4, c + clen - 4))
                elif mtype != 0:
                    yield mtype, s, msize
                s += msize

    def links(self, addr):
        out = {}
        for mtype, s, _ in self.messages(addr):
            if mtype != 0x06:
                continue
            ver, fl = self.raw[s], self.raw[s + 1]
            if ver != 1:
                raise ValueError("link message version")
            q = s + 2
            ltype = 0
            if fl & 0x08:
                ltype = self.raw[q]
                q += 1
            if fl & 0x04:
                q += 8                            # creation order
            if fl & 0x10:
                q += 1                            # name character set
            w = 1 << (fl & 3)
            nlen = int.from_bytes(self.raw[q:q + w], "little")
            q += w
            name = self.raw[q:q + nlen].decode("utf-8")
            q += nlen
            if ltype == 0:                        # hard link
                out[name] = self.u("Q", q)[0]
        return out

    def dataset(self, addr):
        dims = dtype_ok = data = None
        for mtype, s, _ in self.messages(addr):
            if mtype == 0x01:                     # dataspace
                ver = self.raw[s]
                if ver == 1:
                    rank, fl = self.raw[s + 1], self.raw[s + 2]
                    q = s + 8
                elif ver == 2:
                    rank, fl = self.raw[s + 1], self.raw[s + 2]
                    q = s + 4
                else:
                    raise ValueError("dataspace version")
                dims = list(self.u(f"{rank}Q", q)) if rank else []
            elif mtype == 0x03:                   # datatype
                cls, ver = self.raw[s] & 0x0F, self.raw[s] >> 4
                bits0 = self.raw[s + 1]
                size = self.u("I", s + 4)[0]
                if cls != 1 or size != 8 or (bits0 & 1):
                    raise ValueError("only little-endian IEEE float64 datasets are supported")
                dtype_ok = True
            elif mtype == 0x08:                   # data layout
                ver, cls = self.raw[s], self.raw[s + 1]
                if ver not in (3, 4):
                    raise ValueError("layout version")
                if cls == 0:                      # compact
                    n = self.u("H", s + 2)[0]
                    data = self.raw[s + 4:s + 4 + n]
                elif cls == 1:                    # contiguous
                    a, n = self.u("QQ", s + 2)
                    data = b"" if a == _UNDEF else self.raw[self.base + a:self.base + a + n]
                else:
                    raise ValueError("chunked/virtual layouts are not supported")
        if dims is None or not dtype_ok or data is None:
            raise ValueError(f"object at {addr:#x} is not a plain float64 dataset")
        return np.frombuffer(data, dtype="<f8").reshape(dims).astype(np.float64)


def read(path_or_bytes, names=None) -> dict:
    """-> {dataset name: float64 ndarray} for the root group's datasets (or `names`)."""
    raw = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    f = _File(bytes(raw))
    links = f.links(f.root)
    want = links if names is None else {n: links[n] for n in names}
    return {n: f.dataset(a) for n, a in want.items()}
