"""Rating files: the reference's env.readCsvFile[(Int, Int, Double)](path) (DSGDforMF.scala:72)
and MovieLens u.data, parsed by libmfhip's multi-threaded reader (mf_read_ratings)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


def read_ratings(path: str, delimiter: str = ",", skip_lines: int = 0):
    """(users int32, items int32, ratings float64) of a "user<d>item<d>rating[<d>...]" file.
    delimiter: "," (Flink's readCsvFile default), "\t" (u.data) or "" for any run of spaces,
    tabs or commas; extra fields (u.data's timestamp) are ignored; a bad line raises MFError."""
    lib = L.lib()
    d = C.c_char(delimiter.encode()[:1] or b"\0")
    n = C.c_int64(0)
    L.check(lib.mf_read_ratings(path.encode(), d, skip_lines, None, None, None, 0, C.byref(n)))
    u = np.empty(n.value, np.int32)
    i = np.empty(n.value, np.int32)
    r = np.empty(n.value, np.float64)
    got = C.c_int64(0)
    L.check(lib.mf_read_ratings(path.encode(), d, skip_lines, L.ptr(u, C.c_int32), L.ptr(i, C.c_int32),
                                L.ptr(r, C.c_double), n.value, C.byref(got)))
    return u, i, r
