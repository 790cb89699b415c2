"""Reader for R's save() files (RDX2 / XDR serialization) -- the tick data of
the reference's Tayal (2009) replication (tayal2009/data/<SYM>/<date>.<SYM>.RData,
loaded with `load()` at tayal2009/main.R:47-58, one xts per file).

A data-only decoder of R's serialization format version 2: it materialises
vectors (logical, integer, double, character, list), pairlists, symbols and
attributes, and refuses anything that would carry code (closures, promises,
bytecode, environments other than the global/base/empty markers).  Nothing is
evaluated.  Feeds the feature extractor:

    price, size, time = load_ticks([...paths...])   # tdata <- na.omit(series[, 1:2])
    legs = hhmm_amd.features.extract_features(price, size, time, 0.25)
"""
import gzip
import struct

import numpy as np

NILVALUE, GLOBALENV, UNBOUNDVALUE, MISSINGARG, BASENAMESPACE = 254, 253, 252, 251, 250
EMPTYENV, BASEENV, REFSXP = 242, 241, 255
SYMSXP, LISTSXP, CHARSXP, LGLSXP, INTSXP, REALSXP, CPLXSXP, STRSXP, VECSXP = 1, 2, 9, 10, 13, 14, 15, 16, 19
NA_INTEGER = -(2 ** 31)


class RObject:
    """A decoded R value: `value` (numpy array / list / str / None) plus `attributes`."""

    def __init__(self, rtype, value, attributes=None):
        self.rtype = rtype
        self.value = value
        self.attributes = attributes or {}

    def attr(self, name, default=None):
        a = self.attributes.get(name)
        return default if a is None else a.value

    def __repr__(self):
        return f"RObject(type={self.rtype}, attrs={list(self.attributes)})"


class _Reader:
    def __init__(self, buf):
        self.b = buf
        self.i = 0
        self.refs = []

    def int(self):
        v = struct.unpack_from(">i", self.b, self.i)[0]
        self.i += 4
        return v

    def length(self):
        n = self.int()
        if n == -1:
            hi, lo = self.int(), self.int()
            n = (hi << 32) + (lo & 0xFFFFFFFF)
        return n

    def item(self):
        flags = self.int()
        t = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == NILVALUE:
            return None
        if t in (GLOBALENV, EMPTYENV, BASEENV, BASENAMESPACE, UNBOUNDVALUE, MISSINGARG):
            return RObject(t, None)
        if t == REFSXP:
            k = flags >> 8
            if k == 0:
                k = self.int()
            return self.refs[k - 1]
        if t == SYMSXP:
            name = self.item()
            sym = RObject(SYMSXP, name.value if isinstance(name, RObject) else name)
            self.refs.append(sym)
            return sym
        if t == LISTSXP:
            return self._pairlist(has_attr, has_tag)
        if t == CHARSXP:
            n = self.int()
            if n == -1:
                return RObject(CHARSXP, None)
            s = self.b[self.i:self.i + n].decode("utf-8", "replace")
            self.i += n
            return RObject(CHARSXP, s)
        if t in (LGLSXP, INTSXP):
            n = self.length()
            v = np.frombuffer(self.b, dtype=">i4", count=n, offset=self.i).astype(np.int32)
            self.i += 4 * n
            obj = RObject(t, v)
        elif t == REALSXP:
            n = self.length()
            v = np.frombuffer(self.b, dtype=">f8", count=n, offset=self.i).astype(np.float64)
            self.i += 8 * n
            obj = RObject(t, v)
        elif t == CPLXSXP:
            n = self.length()
            v = np.frombuffer(self.b, dtype=">f8", count=2 * n, offset=self.i).astype(np.float64)
            self.i += 16 * n
            obj = RObject(t, v[0::2] + 1j * v[1::2])
        elif t == STRSXP:
            n = self.length()
            obj = RObject(t, [self.item().value for _ in range(n)])
        elif t == VECSXP:
            n = self.length()
            obj = RObject(t, [self.item() for _ in range(n)])
        else:
            raise ValueError(f"R type {t} is not data (closure, environment, bytecode, ...): refusing")
        if has_attr:
            obj.attributes = self._attributes(self.item())
        return obj

    def _pairlist(self, has_attr, has_tag):
        """A pairlist as an ordered list of (tag, value); iterative over the cdr chain."""
        items = []
        attrs = None
        while True:
            if has_attr:
                attrs = self.item()
            tag = self.item() if has_tag else None
            car = self.item()
            items.append((tag.value if isinstance(tag, RObject) else None, car))
            flags = self.int()
            t = flags & 0xFF
            if t == NILVALUE:
                break
            if t != LISTSXP:
                raise ValueError(f"unexpected pairlist tail of type {t}")
            has_attr = bool(flags & (1 << 9))
            has_tag = bool(flags & (1 << 10))
        obj = RObject(LISTSXP, items)
        if attrs is not None:
            obj.attributes = self._attributes(attrs)
        return obj

    @staticmethod
    def _attributes(pl):
        if pl is None:
            return {}
        return {tag: val for tag, val in pl.value}


def read_rdata(path):
    """{name: RObject} of an .RData file written by save() (gzip or plain)."""
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    if raw[:5] != b"RDX2\n":
        raise ValueError(f"{path}: not an RDX2 save file")
    if raw[5:7] != b"X\n":
        raise ValueError(f"{path}: only the XDR serialization is supported")
    r = _Reader(raw)
    r.i = 7
    version = r.int()
    r.int()  # writer R version
    r.int()  # minimal reader version
    if version != 2:
        raise ValueError(f"{path}: serialization version {version} (expected 2)")
    top = r.item()
    return {tag: val for tag, val in top.value}


def xts_columns(obj):
    """(index seconds, {column name: values}) of an xts matrix object."""
    dim = obj.attr("dim")
    nrow, ncol = (int(dim[0]), int(dim[1])) if dim is not None else (len(obj.value), 1)
    names = [f"V{j + 1}" for j in range(ncol)]
    dn = obj.attr("dimnames")
    if dn is not None and len(dn) > 1 and dn[1] is not None:
        names = list(dn[1].value)
    vals = np.asarray(obj.value, dtype=np.float64).reshape(ncol, nrow).T
    index = obj.attr("index")
    if index is None:
        raise ValueError("not an xts object (no index attribute)")
    return np.asarray(index, dtype=np.float64), {n: vals[:, j] for j, n in enumerate(names)}


def load_ticks(paths):
    """tdata <- na.omit(do.call(rbind, lapply(files, load))[, 1:2]) (tayal2009/main.R:47-58):
    returns (price, size, time) of the concatenated files, rows with NA in the
    first two columns dropped."""
    if isinstance(paths, (str, bytes)) or hasattr(paths, "__fspath__"):
        paths = [paths]
    ts, cols = [], []
    for p in paths:
        for obj in read_rdata(p).values():
            idx, c = xts_columns(obj)
            v = list(c.values())
            ts.append(idx)
            cols.append(np.stack([v[0], v[1]], axis=1))
    t = np.concatenate(ts)
    m = np.concatenate(cols)
    order = np.argsort(t, kind="stable")  # rbind.xts merges by index
    t, m = t[order], m[order]
    keep = ~np.isnan(m).any(axis=1)
    return m[keep, 0].copy(), m[keep, 1].copy(), t[keep].copy()
