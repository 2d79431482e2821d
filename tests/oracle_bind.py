"""ctypes binding of the CPU restatement (oracle/) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from imsame_amd.abi import Params, ReadResult, RESULT_DTYPE

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
# IMSAME_ORACLE_LIB / _BIN: other builds of the same source (scripts/sanitize.sh)
LIB = os.environ.get("IMSAME_ORACLE_LIB") or os.path.join(ORACLE_DIR, "build", "liboracle.so")
BIN = os.environ.get("IMSAME_ORACLE_BIN") or os.path.join(ORACLE_DIR, "build", "imsame_oracle")


class NwOut(C.Structure):
    _fields_ = [("score", C.c_int64), ("bx", C.c_uint64), ("by", C.c_uint64),
                ("length", C.c_uint64), ("identities", C.c_uint64), ("igaps", C.c_uint64),
                ("egaps", C.c_uint64), ("head_x", C.c_uint64), ("head_y", C.c_uint64)]


class UgOut(C.Structure):
    _fields_ = [("x_start", C.c_uint64), ("y_start", C.c_uint64), ("t_len", C.c_uint64),
                ("raw", C.c_uint64), ("e_value", C.c_longdouble), ("e_value_d", C.c_double),
                ("pass_", C.c_int)]


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)


def _p(a, t=C.c_uint8):
    return a.ctypes.data_as(C.POINTER(t))


class Oracle:
    _inst = None

    @classmethod
    def load(cls, build=False):
        if cls._inst is None:
            if (build and not os.environ.get("IMSAME_ORACLE_LIB")) or not os.path.exists(LIB):
                build_oracle()
            cls._inst = cls(C.CDLL(LIB))
        return cls._inst

    def __init__(self, lib):
        self.lib = lib
        lib.or_nw.argtypes = [C.c_char_p, C.c_uint64, C.c_char_p, C.c_uint64, C.c_int64, C.c_int64,
                              C.POINTER(NwOut), C.c_char_p, C.c_uint64, C.POINTER(C.c_uint64)]
        lib.or_ungapped.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                    C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, C.c_double,
                                    C.POINTER(UgOut)]
        lib.or_align.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                 C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                 C.POINTER(Params), C.c_uint64, C.c_void_p, C.POINTER(C.c_uint64)]
        lib.or_align_windows.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                         C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                         C.POINTER(Params), C.c_uint64, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.POINTER(C.c_uint64)]
        lib.or_revcomp.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        lib.or_params_default.argtypes = [C.POINTER(Params)]

    def params(self, **kw):
        p = Params()
        self.lib.or_params_default(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def nw(self, X, Y, igap=-5, egap=-2, text=True):
        X = X.encode() if isinstance(X, str) else X
        Y = Y.encode() if isinstance(Y, str) else Y
        o = NwOut()
        cap = 64 + 6 * (len(X) + len(Y)) * 3 if text else 0
        buf = C.create_string_buffer(cap + 1) if text else None
        tl = C.c_uint64()
        rc = self.lib.or_nw(X, len(X), Y, len(Y), igap, egap, C.byref(o), buf, cap, C.byref(tl))
        assert rc == 0
        d = {k: getattr(o, k) for k, _ in NwOut._fields_}
        if text:
            d["text"] = buf.raw[:tl.value]
        return d

    def ungapped(self, db, db_start, q, q_start, pos_db, pos_q, read, dbseq, min_e=-1.0):
        db = np.ascontiguousarray(db, dtype=np.uint8)
        q = np.ascontiguousarray(q, dtype=np.uint8)
        dbs = np.ascontiguousarray(db_start, dtype=np.uint64)
        qs = np.ascontiguousarray(q_start, dtype=np.uint64)
        o = UgOut()
        self.lib.or_ungapped(db.ctypes.data, len(db), dbs.ctypes.data, len(dbs),
                             q.ctypes.data, len(q), qs.ctypes.data, len(qs),
                             pos_db, pos_q, read, dbseq, min_e, C.byref(o))
        return o

    def align(self, db, db_start, q, q_start, params=None, n_threads=1, db_brk=None):
        """Per-read results (numpy RESULT_DTYPE array) for all reads."""
        db = np.ascontiguousarray(db, dtype=np.uint8)
        q = np.ascontiguousarray(q, dtype=np.uint8)
        dbs = np.ascontiguousarray(db_start, dtype=np.uint64)
        qs = np.ascontiguousarray(q_start, dtype=np.uint64)
        p = params if params is not None else self.params()
        res = np.zeros(len(qs), dtype=RESULT_DTYPE)
        er = C.c_uint64()
        brk = None if db_brk is None else np.ascontiguousarray(db_brk, dtype=np.uint8)
        rc = self.lib.or_align(db.ctypes.data, len(db), dbs.ctypes.data, len(dbs),
                               None if brk is None else brk.ctypes.data,
                               q.ctypes.data, len(q), qs.ctypes.data, len(qs),
                               C.byref(p), n_threads, res.ctypes.data, C.byref(er))
        return rc, res, er.value

    def align_windows(self, db, db_start, q, q_start, windows, params=None, n_threads=1, db_brk=None):
        """Per-read results of the reads of windows [(a, b), ...] of the whole
        query (its chunk heads), without aligning the rest: (rc, [res of each
        window], err)."""
        db = np.ascontiguousarray(db, dtype=np.uint8)
        q = np.ascontiguousarray(q, dtype=np.uint8)
        dbs = np.ascontiguousarray(db_start, dtype=np.uint64)
        qs = np.ascontiguousarray(q_start, dtype=np.uint64)
        p = params if params is not None else self.params()
        res = np.zeros(len(qs), dtype=RESULT_DTYPE)
        wf = np.array([w[0] for w in windows], dtype=np.uint64)
        wt = np.array([w[1] for w in windows], dtype=np.uint64)
        er = C.c_uint64()
        brk = None if db_brk is None else np.ascontiguousarray(db_brk, dtype=np.uint8)
        rc = self.lib.or_align_windows(db.ctypes.data, len(db), dbs.ctypes.data, len(dbs),
                                       None if brk is None else brk.ctypes.data,
                                       q.ctypes.data, len(q), qs.ctypes.data, len(qs),
                                       C.byref(p), n_threads, len(windows), wf.ctypes.data, wt.ctypes.data,
                                       res.ctypes.data, C.byref(er))
        return rc, [res[a:b] for a, b in windows], er.value

    def revcomp(self, data):
        src = np.frombuffer(data, dtype=np.uint8)
        cap = len(data) + data.count(b">") + 2
        out = np.zeros(cap, dtype=np.uint8)
        ol = C.c_uint64()
        rc = self.lib.or_revcomp(src.ctypes.data if len(src) else None, len(src), out.ctypes.data, cap,
                                 C.byref(ol))
        if rc != 0:      # '>' inside headers duplicates bytes: size reported back
            out = np.zeros(ol.value, dtype=np.uint8)
            rc = self.lib.or_revcomp(src.ctypes.data, len(src), out.ctypes.data, ol.value, C.byref(ol))
        assert rc == 0
        return out[:ol.value].tobytes()

    @staticmethod
    def run_cli(args, timeout=600):
        build_oracle() if not os.path.exists(BIN) else None
        return subprocess.run([BIN] + list(args), stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              timeout=timeout)
