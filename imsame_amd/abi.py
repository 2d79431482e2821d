"""ctypes mirror of include/imsame_dev.h (the C-ABI boundary).

Kept in lock-step with the header; tests/test_abi.py checks sizes/offsets
against the compiled library.
"""
import ctypes as C

import numpy as np

IMSAME_OK = 0
IMSAME_E_HIP = -1
IMSAME_E_OOM = -2
IMSAME_E_READ_TOO_LONG = -3
IMSAME_E_ARG = -4
IMSAME_E_RANGE = -5
IMSAME_E_PATHS = -6
IMSAME_E_STATE = -7

FIXED_K = 12
POINT = 4
MAX_READ_SIZE = 3000
ALIGN_LEN = 60

MOVE_DIAG, MOVE_UP, MOVE_LEFT = 0, 1, 2
LAUNCH_STATS = 64        # IMSAME_LAUNCH_STATS


class Params(C.Structure):
    _fields_ = [
        ("min_e", C.c_longdouble),
        ("min_coverage", C.c_longdouble),
        ("min_identity", C.c_longdouble),
        ("igap", C.c_int64),
        ("egap", C.c_int64),
        ("max_read_size", C.c_uint64),
        ("want_paths", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class ReadResult(C.Structure):
    _fields_ = [
        ("db_seq", C.c_uint64),
        ("score", C.c_int64),
        ("bx", C.c_uint32), ("by", C.c_uint32),
        ("length", C.c_uint32), ("identities", C.c_uint32),
        ("igaps", C.c_uint32), ("egaps", C.c_uint32),
        ("head_x", C.c_uint32), ("head_y", C.c_uint32),
        ("ylen", C.c_uint32), ("status", C.c_uint32),
        ("path_off", C.c_uint32), ("path_len", C.c_uint32),
    ]


# numpy view of an imsame_read_result array
RESULT_DTYPE = np.dtype([
    ("db_seq", "<u8"), ("score", "<i8"), ("bx", "<u4"), ("by", "<u4"),
    ("length", "<u4"), ("identities", "<u4"), ("igaps", "<u4"), ("egaps", "<u4"),
    ("head_x", "<u4"), ("head_y", "<u4"), ("ylen", "<u4"), ("status", "<u4"),
    ("path_off", "<u4"), ("path_len", "<u4"),
])
assert RESULT_DTYPE.itemsize == 64 == C.sizeof(ReadResult)

# fields that must be bit-identical between the device and the reference
PARITY_FIELDS = ("status", "db_seq", "score", "bx", "by", "length", "identities",
                 "igaps", "egaps", "head_x", "head_y", "ylen")


class Stats(C.Structure):
    _fields_ = [
        ("n_reads", C.c_uint64), ("n_accepted", C.c_uint64), ("n_nw", C.c_uint64),
        ("nw_cells", C.c_uint64), ("n_hits", C.c_uint64), ("rounds", C.c_uint64),
        ("err_read", C.c_uint64), ("err_dbseq", C.c_uint64),
        ("ms_seed", C.c_double), ("ms_nw", C.c_double), ("ms_total", C.c_double),
        ("nw_launch_ms", C.c_double), ("nw_launches", C.c_uint64), ("nw_bytes", C.c_uint64),
        ("launch_cand", C.c_uint64 * LAUNCH_STATS), ("launch_ms", C.c_double * LAUNCH_STATS),
        ("n_rewalk", C.c_uint64), ("ms_setup", C.c_double), ("ms_d2h", C.c_double),
        ("ms_nw_busy", C.c_double), ("lanes", C.c_uint64), ("nw_redo", C.c_uint64),
        ("launch_pk", C.c_uint64), ("nw_win", C.c_uint64), ("ms_nw_first", C.c_double),
        ("ms_nw_last", C.c_double), ("launch_k5", C.c_uint64), ("launch_np", C.c_uint64),
        ("launch_k19", C.c_uint64), ("launch_nwp", C.c_uint64), ("nw_fallback", C.c_uint64),
        ("seed_windows", C.c_uint64), ("seed_entries", C.c_uint64), ("seed_ext_chunks", C.c_uint64),
        ("nw_spec_waste", C.c_uint64), ("launch_k3", C.c_uint64),
    ]

    def as_dict(self):
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if k in ("launch_cand", "launch_ms") else v
        k = min(self.nw_launches, LAUNCH_STATS)
        d["launch_cand"], d["launch_ms"] = d["launch_cand"][:k], d["launch_ms"][:k]
        return d


def default_params():
    """Reference defaults (IMSAME.c:44-49): min_e = 1/powl(10,20) is not a
    Python float -- callers needing it exactly use the library's
    imsame_params_default(); this helper is for the oracle, which applies
    the same default when min_e is passed as a negative sentinel."""
    p = Params()
    p.min_e = C.c_longdouble(1e-20)
    p.min_coverage = 0.5
    p.min_identity = 0.5
    p.igap = -5
    p.egap = -2
    p.max_read_size = MAX_READ_SIZE
    p.want_paths = 0
    return p
