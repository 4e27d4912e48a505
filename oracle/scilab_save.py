"""Reader for the Scilab 5 binary ``save`` format (test infrastructure only).

The GLONASS SoftGNSS receivers end their tracking run with
``save('trackingResults.dat', trackResults, settings, acqResults, channel)``
(``SCI/GLONASS/L1/postProcessing.sce:143``, the same line in ``L2``). The two
files the reference ships are the only recorded output of the Scilab float
tracking loop (``tracking.sci``), so they pin ``sgt_oracle`` and ``sgt.hip``'s
loop half (tests/test_sgt_trackres.py). No Scilab is installed in the image;
this module decodes the format directly. It executes nothing from the file: it
reads fixed-width integers, doubles and character codes.

Layout, as the file itself shows (all little-endian, no alignment padding):

* A variable is a 24-byte name followed by its value. The name is six int32
  words, each the arithmetic sum ``c0 + 256 c1 + 65536 c2 + 2^24 c3`` of four
  Scilab character codes (codes may be negative for upper case, so decoding
  carries the borrow into the next byte). Code 40 is the blank padding.
* Scilab character codes: ``0-9`` -> 0..9, ``a-z`` -> 10..35, upper case is the
  negated lower case code; the punctuation table below covers the rest.
* A value starts with an int32 type word:
    - 1  real/complex matrix: m, n, it, then m*n doubles (and m*n imaginary
      doubles when it == 1), column-major;
    - 4  boolean matrix: m, n, then m*n int32;
    - 8  integer matrix: m, n, it (1/2/4 signed, 11/12/14 unsigned bytes), then
      the m*n values packed at their own width;
    - 10 string matrix: m, n, 0, m*n+1 one-based offsets, then one int32
      character code per character;
    - 15/16/17 list / tlist / mlist: n, n+1 offsets, then the n items in order.
  The offsets of lists and strings are the in-memory stack offsets (units of
  doubles); the file stores items back to back, so the reader walks them.
* A Scilab ``struct`` is an mlist whose first item is the string row
  ``['st', 'dims', field names...]`` and whose second item is an int32 ``dims``
  matrix; for a 1x1 struct each further item is the field value, for a larger
  struct each is a list of the per-element values.
"""
import numpy as np

_PUNCT = {36: "_", 37: "#", 38: "!", 39: "$", 40: " ", 41: "(", 42: ")", 43: ";",
          44: ":", 45: "+", 46: "-", 47: "*", 48: "/", 49: "\\", 50: "=", 51: ".",
          52: ",", 53: "'", 54: "[", 55: "]", 56: "%", 57: "|", 58: "&", 59: "<",
          60: ">", 61: "~", 62: "^"}


def _char(c):
    if 0 <= c <= 9:
        return chr(ord("0") + c)
    if 10 <= c <= 35:
        return chr(ord("a") + c - 10)
    if -35 <= c <= -10:
        return chr(ord("A") - c - 10)
    if c in _PUNCT:
        return _PUNCT[c]
    if -c in _PUNCT:      # shifted punctuation: Scilab's alternate codes
        return _PUNCT[-c]
    return "?"


def _name(raw):
    out = []
    for w in np.frombuffer(raw, dtype="<i4").tolist():
        w &= 0xFFFFFFFF
        codes, carry = [], 0
        for k in range(4):
            c = ((w >> (8 * k)) & 0xFF) + carry
            carry = 0
            if c > 127:
                c -= 256
                carry = 1
            codes.append(c)
        out.extend(codes)
    s = "".join(_char(c) for c in out)
    return s.rstrip()


class ScilabStruct(dict):
    """A 1x1 Scilab struct, or one element of a struct array."""


class _Reader:
    def __init__(self, data):
        self.b = data
        self.o = 0

    def i32(self, n=1):
        v = np.frombuffer(self.b, dtype="<i4", count=n, offset=self.o)
        self.o += 4 * n
        return v

    def f64(self, n):
        v = np.frombuffer(self.b, dtype="<f8", count=n, offset=self.o)
        self.o += 8 * n
        return v

    def value(self):
        t = int(self.i32()[0])
        if t == 1:
            m, n, it = (int(x) for x in self.i32(3))
            re = self.f64(m * n).reshape((n, m)).T
            if it:
                im = self.f64(m * n).reshape((n, m)).T
                return re + 1j * im
            return re.copy()
        if t == 4:
            m, n = (int(x) for x in self.i32(2))
            return (self.i32(m * n).reshape((n, m)).T != 0)
        if t == 8:
            m, n, it = (int(x) for x in self.i32(3))
            dt = {1: "<i1", 2: "<i2", 4: "<i4", 11: "<u1", 12: "<u2", 14: "<u4"}[it]
            w = np.dtype(dt).itemsize
            v = np.frombuffer(self.b, dtype=dt, count=m * n, offset=self.o)
            self.o += w * m * n
            return v.reshape((n, m)).T.copy()
        if t == 10:
            m, n, _ = (int(x) for x in self.i32(3))
            offs = self.i32(m * n + 1)
            codes = self.i32(int(offs[-1]) - 1)
            strs = ["".join(_char(int(c)) for c in codes[offs[k] - 1:offs[k + 1] - 1])
                    for k in range(m * n)]
            if m * n == 1:
                return strs[0]
            return np.array(strs, dtype=object).reshape((n, m)).T
        if t in (15, 16, 17):
            n = int(self.i32()[0])
            self.i32(n + 1)
            items = [self.value() for _ in range(n)]
            if t == 17 and items and isinstance(items[0], np.ndarray) and \
                    items[0].size >= 2 and items[0].flat[0] == "st":
                return _struct(items)
            return items
        raise ValueError(f"unsupported Scilab type {t} at byte {self.o - 4}")


def _struct(items):
    fields = [str(f) for f in items[0].flat[2:]]
    dims = np.asarray(items[1]).ravel().astype(int)
    count = int(np.prod(dims))
    if count == 1:
        s = ScilabStruct(zip(fields, items[2:]))
        s.dims = tuple(dims)
        return s
    elems = []
    for k in range(count):
        elems.append(ScilabStruct((f, items[2 + j][k]) for j, f in enumerate(fields)))
    return elems


def load(path):
    """All variables of a Scilab 5 binary save file, in file order."""
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    out = {}
    while r.o + 24 <= len(data):
        name = _name(data[r.o:r.o + 24])
        r.o += 24
        out[name] = r.value()
    return out
