"""ctypes binding of the CPU wave emulator (tests/emu/) -- TEST INFRASTRUCTURE.

It runs the device kernel SOURCE (imsame_amd/csrc/*_kernel.hip) on host
threads, so the kernels' logic is checked in the CPU suite; the GPU suite
checks the compiled kernels themselves.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from imsame_amd.abi import Params, Stats, RESULT_DTYPE

HERE = os.path.dirname(os.path.abspath(__file__))
EMU_DIR = os.path.join(HERE, "emu")
LIB = os.environ.get("IMSAME_EMU_LIB") or os.path.join(EMU_DIR, "build", "libwave_emu.so")   # (scripts/sanitize.sh)


class Emu:
    _inst = None

    @classmethod
    def load(cls):
        if cls._inst is None:
            subprocess.run(["make", "-s", "-C", EMU_DIR], check=True)
            cls._inst = cls(C.CDLL(LIB))
        return cls._inst

    def __init__(self, lib):
        self.lib = lib
        lib.emu_nw_pairs.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                     C.POINTER(Params), C.c_void_p, C.c_void_p, C.c_uint64,
                                     C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)]
        lib.emu_align.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p,
                                  C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                  C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(Params),
                                  C.c_void_p, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64),
                                  C.POINTER(Stats)]

    def nw_pairs(self, X, Y, params, paths_cap=0):
        xs = np.frombuffer(b"".join(X), dtype=np.uint8).copy()
        ys = np.frombuffer(b"".join(Y), dtype=np.uint8).copy()
        xst = np.cumsum([0] + [len(x) for x in X]).astype(np.uint64)
        yst = np.cumsum([0] + [len(y) for y in Y]).astype(np.uint64)
        res = np.zeros(len(X), dtype=RESULT_DTYPE)
        paths = np.zeros(max(1, paths_cap), dtype=np.uint32)
        used = C.c_uint64()
        flags = C.c_uint32()
        rc = self.lib.emu_nw_pairs(xs.ctypes.data, xst.ctypes.data, ys.ctypes.data, yst.ctypes.data, len(X),
                                   C.byref(params), res.ctypes.data, paths.ctypes.data, paths_cap,
                                   C.byref(used), C.byref(flags))
        return rc, res, paths[:used.value], flags.value

    def align(self, db, db_start, q, q_start, params, n_threads=1, read_from=0, read_to=None,
              db_brk=None, paths_cap=0):
        db = np.ascontiguousarray(db, dtype=np.uint8)
        q = np.ascontiguousarray(q, dtype=np.uint8)
        dbs = np.ascontiguousarray(db_start, dtype=np.uint64)
        qs = np.ascontiguousarray(q_start, dtype=np.uint64)
        read_to = len(qs) if read_to is None else read_to
        res = np.zeros(read_to - read_from, dtype=RESULT_DTYPE)
        paths = np.zeros(max(1, paths_cap), dtype=np.uint32)
        used = C.c_uint64()
        st = Stats()
        brk = None if db_brk is None else np.ascontiguousarray(db_brk, dtype=np.uint8)
        rc = self.lib.emu_align(db.ctypes.data, len(db), dbs.ctypes.data, len(dbs),
                                None if brk is None else brk.ctypes.data,
                                q.ctypes.data, len(q), qs.ctypes.data, len(qs), read_from, read_to,
                                n_threads, C.byref(params), res.ctypes.data, paths.ctypes.data, paths_cap,
                                C.byref(used), C.byref(st))
        return rc, res, paths[:used.value], st
