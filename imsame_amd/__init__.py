"""imsame_amd -- MI355X-native IMSAME seed-and-extend path.

Python mirror of the C-ABI boundary (include/imsame_dev.h).  The reference
(Bitlab-UMA/IMSAME) is a C program; its seam for this path is the pthread
worker computeAlignmentsByThread (alignmentFunctions.c:43) fed by the 12-mer
index built in main (IMSAME.c:194-289).  Here:

    dev = Device(0)                         # imsame_dev_open
    dev.index(db_seq, db_starts, db_brk)    # replaces IMSAME.c:232-281
    dev.set_query(q_seq, q_starts)
    res, paths, stats = dev.align(n_threads=T, params=dev.params())
                                            # replaces T x computeAlignmentsByThread

Every call runs on the GPU through libimsame_dev.so; there is no CPU
fallback -- a missing library or device raises ImsameError.
"""
import ctypes as C
import os

import numpy as np

from . import abi
from .abi import Params, Stats, RESULT_DTYPE, PARITY_FIELDS  # noqa: F401

# Lanes: the library runs one alignment lane per two hardware queues, read
# from GPU_MAX_HW_QUEUES as the HIP runtime saw it (imsame_dev.hip:hw_queues;
# the library itself never sets it).  HIP's default is 4 (2 lanes, where 8
# queues give 4 lanes and 1-2 % more at C2), so a Python host that has not
# chosen asks for 8 here -- effective only when nothing in this process has
# started HIP yet (the CLI and bench.py set it at start-up for the same
# reason).  Results never depend on it.  This changes the variable for the
# whole process (any HIP user started later sees it): IMSAME_NO_HWQ_DEFAULT=1
# leaves the environment alone (the library then runs the lanes HIP's 4
# queues allow), see INTEGRATION.md.
if not os.environ.get("GPU_MAX_HW_QUEUES") and not os.environ.get("IMSAME_NO_HWQ_DEFAULT"):
    os.environ["GPU_MAX_HW_QUEUES"] = "8"

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DEV = os.environ.get("IMSAME_LIB_DEV") or os.path.join(HERE, "lib", "libimsame_dev.so")
LIB_HOST = os.environ.get("IMSAME_LIB_HOST") or os.path.join(HERE, "lib", "libimsame_host.so")
CLI = os.path.join(HERE, "bin", "imsame")
FLAG_NW32 = 1          # imsame_params.flags: force the int32 NW kernel (include/imsame_dev.h)
FLAG_NW16 = 2          # ... or the packed int16 kernel for every launch it fits, however small
FLAG_NW16_ONEPASS = 4  # ... the packed kernel in one pass (default: score sweep + traceback band)

_lib = None
_host = None
# imsame_part_fn (include/imsame_dev.h)
PART_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_uint64, C.c_uint64, C.c_int, C.c_uint64, C.POINTER(C.c_uint32),
                      C.c_uint64)


class ImsameError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = _strerror(code) if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


def _strerror(code):
    return _lib.imsame_strerror(code).decode()


def lib():
    """Load libimsame_dev.so (built by __graft_entry__.build / csrc/Makefile)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_DEV):
            raise ImsameError(abi.IMSAME_E_STATE, f"{LIB_DEV} missing: run __graft_entry__.build()")
        L = C.CDLL(LIB_DEV)
        vp, u64 = C.c_void_p, C.c_uint64
        L.imsame_strerror.restype = C.c_char_p
        L.imsame_strerror.argtypes = [C.c_int]
        L.imsame_params_default.argtypes = [C.POINTER(Params)]
        L.imsame_dev_open.argtypes = [C.c_int, C.POINTER(vp)]
        L.imsame_dev_close.argtypes = [vp]
        L.imsame_dev_index.argtypes = [vp, vp, u64, vp, u64, vp]
        L.imsame_dev_set_query.argtypes = [vp, vp, u64, vp, u64]
        L.imsame_dev_set_query_range.argtypes = [vp, vp, u64, vp, u64, u64, u64]
        L.imsame_dev_set_query_range_async.argtypes = [vp, vp, u64, vp, u64, u64, u64]
        L.imsame_dev_sync.argtypes = [vp]
        L.imsame_dev_fetch_paths.argtypes = [vp, vp, u64, C.POINTER(u64)]
        L.imsame_host_alloc.restype = vp
        L.imsame_host_alloc.argtypes = [u64]
        L.imsame_host_free.argtypes = [vp]
        L.imsame_dev_align.argtypes = [vp, u64, u64, u64, C.POINTER(Params), vp, vp, u64, C.POINTER(u64),
                                       C.POINTER(Stats)]
        L.imsame_dev_align_parts.argtypes = [vp, u64, u64, u64, C.POINTER(Params), vp, PART_FN, vp,
                                             C.POINTER(Stats)]
        L.imsame_dev_align_windows.argtypes = [vp, u64, u64, u64, C.POINTER(Params), u64, vp, vp, vp, vp, vp, u64,
                                               C.POINTER(u64), C.POINTER(Stats)]
        L.imsame_dev_align_sliced.argtypes = [vp, vp, u64, vp, u64, vp, u64, u64, u64, u64, C.POINTER(Params),
                                              vp, vp, u64, C.POINTER(u64), C.POINTER(u64), C.POINTER(Stats)]
        L.imsame_dev_nw_pairs.argtypes = [vp, vp, vp, vp, vp, u64, C.POINTER(Params), vp, vp, u64,
                                          C.POINTER(u64), C.POINTER(C.c_double)]
        L.imsame_dev_revcomp.argtypes = [vp, vp, u64, vp, u64, C.POINTER(u64)]
        _lib = L
    return _lib


def host_lib():
    global _host
    if _host is None:
        H = C.CDLL(LIB_HOST)
        H.host_render.restype = C.c_uint64
        H.host_render.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.POINTER(abi.ReadResult),
                                  C.c_void_p, C.c_void_p]
        _host = H
    return _host


class _Text(C.Structure):
    _fields_ = [("buf", C.c_void_p), ("len", C.c_size_t), ("cap", C.c_size_t)]


def render(X, Y, result_row, path):
    """.align body text of one accepted read (build_alignment text,
    alignmentFunctions.c:230-271) from a device path."""
    H = host_lib()
    rr = abi.ReadResult()
    for k in RESULT_DTYPE.names:
        setattr(rr, k, int(result_row[k]))
    X = np.frombuffer(X, dtype=np.uint8) if isinstance(X, (bytes, bytearray)) else X
    Y = np.frombuffer(Y, dtype=np.uint8) if isinstance(Y, (bytes, bytearray)) else Y
    path = np.ascontiguousarray(path, dtype=np.uint32)
    t = _Text()
    ident = H.host_render(X.ctypes.data, len(X), Y.ctypes.data, len(Y), C.byref(rr),
                          path.ctypes.data if len(path) else None, C.byref(t))
    out = C.string_at(t.buf, t.len)
    C.CDLL(None).free(C.c_void_p(t.buf))
    return out, int(ident)


def _arr(a, dt):
    return np.ascontiguousarray(a, dtype=dt)


class PinnedArray:
    """numpy view of page-locked host memory (imsame_host_alloc): faster
    H2D copies of query shards than pageable memory."""

    def __init__(self, n, dtype=np.uint8):
        self.nbytes = max(int(n) * np.dtype(dtype).itemsize, 1)
        self._p = lib().imsame_host_alloc(self.nbytes)
        if not self._p:
            raise ImsameError(abi.IMSAME_E_OOM, "imsame_host_alloc")
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self._p)).view(dtype)[:n]

    def free(self):
        if getattr(self, "_p", None):
            self.array = None
            lib().imsame_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Device:
    """One HIP device context (imsame_ctx)."""

    def __init__(self, device=0):
        L = lib()
        h = C.c_void_p()
        rc = L.imsame_dev_open(device, C.byref(h))
        if rc:
            raise ImsameError(rc, f"imsame_dev_open({device})")
        self._h = h
        self._keep = []
        self.q_range = (0, 0)

    def close(self):
        if getattr(self, "_h", None):
            lib().imsame_dev_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @staticmethod
    def params(**kw):
        """Reference defaults (IMSAME.c:44-49) updated with kw; igap/egap are
        the negative internal values (CLI "-igap 5" -> igap=-5)."""
        p = Params()
        lib().imsame_params_default(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def index(self, db_seq, db_starts, db_brk=None):
        db_seq, db_starts = _arr(db_seq, np.uint8), _arr(db_starts, np.uint64)
        brk = None if db_brk is None else _arr(db_brk, np.uint8)
        rc = lib().imsame_dev_index(self._h, db_seq.ctypes.data, len(db_seq), db_starts.ctypes.data,
                                    len(db_starts), None if brk is None else brk.ctypes.data)
        if rc:
            raise ImsameError(rc, "imsame_dev_index")

    def set_query(self, q_seq, q_starts, read_from=None, read_to=None, wait=True):
        """Upload the query; with read_from/read_to only that shard's reads
        go to HBM (imsame_dev_set_query_range; chunk heads stay the whole
        query's).  wait=False queues the copies (imsame_dev_set_query_range_async):
        the next align's lanes start as their reads arrive; the arrays must
        be page-locked (PinnedArray) and stay unchanged until that call."""
        q_seq, q_starts = _arr(q_seq, np.uint8), _arr(q_starts, np.uint64)
        a = 0 if read_from is None else read_from
        b = len(q_starts) if read_to is None else read_to
        fn = lib().imsame_dev_set_query_range if wait else lib().imsame_dev_set_query_range_async
        rc = fn(self._h, q_seq.ctypes.data, len(q_seq), q_starts.ctypes.data, len(q_starts), a, b)
        if rc:
            raise ImsameError(rc, "imsame_dev_set_query_range")
        self.n_q = len(q_starts)
        self.q_range = (a, b)
        self._q_keep = None if wait else (q_seq, q_starts)   # alive until the copies are done

    def sync(self):
        """Wait for queued work (an asynchronous query upload)."""
        rc = lib().imsame_dev_sync(self._h)
        if rc:
            raise ImsameError(rc, "imsame_dev_sync")

    def fetch_paths(self, cap):
        """Paths of the last align call (after IMSAME_E_PATHS)."""
        paths = np.zeros(max(cap, 1), dtype=np.uint32)
        used = C.c_uint64()
        rc = lib().imsame_dev_fetch_paths(self._h, paths.ctypes.data, cap, C.byref(used))
        if rc:
            raise ImsameError(rc, "imsame_dev_fetch_paths")
        return paths[:used.value]

    def align(self, read_from=None, read_to=None, n_threads=4, params=None, want_paths=False, paths_cap=None,
              allow_too_long=False, out=None):
        """Per-read results (numpy RESULT_DTYPE) for reads [read_from, read_to)
        (default: the uploaded range).  out: a RESULT_DTYPE array to fill
        (e.g. a PinnedArray's, reused across calls)."""
        read_from = self.q_range[0] if read_from is None else read_from
        read_to = self.q_range[1] if read_to is None else read_to
        p = params if params is not None else self.params()
        p.want_paths = 1 if want_paths else 0
        n = read_to - read_from
        if out is not None:
            if out.dtype != RESULT_DTYPE or len(out) < n or not out.flags.c_contiguous:
                raise ImsameError(abi.IMSAME_E_ARG, "align(out=): RESULT_DTYPE array of >= n rows")
            res = out[:n]
        else:
            res = np.zeros(n, dtype=RESULT_DTYPE)
        cap = (paths_cap if paths_cap is not None else 8 * n + 1024) if want_paths else 0
        st = Stats()
        used = C.c_uint64()
        paths = np.zeros(max(cap, 1), dtype=np.uint32)
        rc = lib().imsame_dev_align(self._h, read_from, read_to, n_threads, C.byref(p), res.ctypes.data,
                                    paths.ctypes.data if want_paths else None, cap, C.byref(used), C.byref(st))
        if rc and not (rc in (abi.IMSAME_E_PATHS, abi.IMSAME_E_READ_TOO_LONG)
                       and (rc == abi.IMSAME_E_PATHS or allow_too_long)):
            raise ImsameError(rc, "imsame_dev_align")
        if want_paths and used.value > cap:       # not copied (E_PATHS or E_READ_TOO_LONG): on the device
            paths = self.fetch_paths(used.value)
        return res, paths[:used.value], st

    def align_parts(self, read_from=None, read_to=None, n_threads=4, params=None, want_paths=False):
        """imsame_dev_align_parts: per-read results plus the parts as the
        library handed them over, in arrival order: [(from, to, status,
        err_read, paths of the part), ...] (each part's path_off index its
        own paths)."""
        read_from = self.q_range[0] if read_from is None else read_from
        read_to = self.q_range[1] if read_to is None else read_to
        p = params if params is not None else self.params()
        p.want_paths = 1 if want_paths else 0
        res = np.zeros(read_to - read_from, dtype=RESULT_DTYPE)
        parts = []

        def got(_user, a, b, status, err, paths, n):      # runs on the library's lane threads
            arr = np.ctypeslib.as_array(paths, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
            parts.append((int(a), int(b), int(status), int(err), arr))

        cb = PART_FN(got)
        st = Stats()
        rc = lib().imsame_dev_align_parts(self._h, read_from, read_to, n_threads, C.byref(p), res.ctypes.data, cb,
                                          None, C.byref(st))
        if rc:
            raise ImsameError(rc, "imsame_dev_align_parts")
        return res, parts, st

    def align_windows(self, ev_db_len, win_cap=None, read_from=None, read_to=None, n_threads=4, params=None,
                      allow_too_long=False, win_start=None):
        """align() on the loaded index as ONE SLICE of a database of
        ev_db_len bases: per-read window caps in, accept windows out
        (imsame_dev_align_windows).  Returns (res, win, stats); db_seq is
        slice-local."""
        read_from = self.q_range[0] if read_from is None else read_from
        read_to = self.q_range[1] if read_to is None else read_to
        p = params if params is not None else self.params()
        p.want_paths = 0
        n = read_to - read_from
        res = np.zeros(n, dtype=RESULT_DTYPE)
        win = np.zeros(n, dtype=np.uint64)
        cap = None if win_cap is None else _arr(win_cap, np.uint64)
        ws = None if win_start is None else _arr(win_start, np.uint64)
        st, used = Stats(), C.c_uint64()
        rc = lib().imsame_dev_align_windows(self._h, read_from, read_to, n_threads, C.byref(p), ev_db_len,
                                            None if ws is None else ws.ctypes.data,
                                            None if cap is None else cap.ctypes.data, res.ctypes.data,
                                            win.ctypes.data, None, 0, C.byref(used), C.byref(st))
        if rc and not (rc == abi.IMSAME_E_READ_TOO_LONG and allow_too_long):
            raise ImsameError(rc, "imsame_dev_align_windows")
        return res, win, st

    def align_sliced(self, db_seq, db_starts, slice_bases, db_brk=None, read_from=None, read_to=None, n_threads=4,
                     params=None, want_paths=False, paths_cap=None):
        """align() against db_seq indexed and searched in slices of at most
        slice_bases bases, one slice's index in HBM at a time
        (imsame_dev_align_sliced).  Returns (res, paths, stats, n_slices)."""
        db_seq, db_starts = _arr(db_seq, np.uint8), _arr(db_starts, np.uint64)
        brk = None if db_brk is None else _arr(db_brk, np.uint8)
        read_from = self.q_range[0] if read_from is None else read_from
        read_to = self.q_range[1] if read_to is None else read_to
        p = params if params is not None else self.params()
        p.want_paths = 1 if want_paths else 0
        n = read_to - read_from
        res = np.zeros(n, dtype=RESULT_DTYPE)
        cap = (paths_cap if paths_cap is not None else 8 * n + 1024) if want_paths else 0
        st, used, ns = Stats(), C.c_uint64(), C.c_uint64()
        paths = np.zeros(max(cap, 1), dtype=np.uint32)
        rc = lib().imsame_dev_align_sliced(self._h, db_seq.ctypes.data, len(db_seq), db_starts.ctypes.data,
                                           len(db_starts), None if brk is None else brk.ctypes.data,
                                           slice_bases, read_from, read_to, n_threads, C.byref(p),
                                           res.ctypes.data, paths.ctypes.data if want_paths else None, cap,
                                           C.byref(used), C.byref(ns), C.byref(st))
        if rc and rc != abi.IMSAME_E_PATHS:
            raise ImsameError(rc, "imsame_dev_align_sliced")
        if want_paths and used.value > cap:
            paths = self.fetch_paths(used.value)
        return res, paths[:used.value], st, ns.value

    def nw_pairs(self, X, Y, params=None, want_paths=False):
        """Unit-level NW + backtrack + acceptance of explicit pairs
        (build_alignment, alignmentFunctions.c:210-274)."""
        p = params if params is not None else self.params()
        p.want_paths = 1 if want_paths else 0
        xs = np.frombuffer(b"".join(X), dtype=np.uint8).copy()
        ys = np.frombuffer(b"".join(Y), dtype=np.uint8).copy()
        xst = np.cumsum([0] + [len(x) for x in X]).astype(np.uint64)
        yst = np.cumsum([0] + [len(y) for y in Y]).astype(np.uint64)
        res = np.zeros(len(X), dtype=RESULT_DTYPE)
        cap = (sum(len(x) + len(y) for x, y in zip(X, Y)) + 16) if want_paths else 0
        paths = np.zeros(max(cap, 1), dtype=np.uint32)
        used = C.c_uint64()
        ms = C.c_double()
        rc = lib().imsame_dev_nw_pairs(self._h, xs.ctypes.data, xst.ctypes.data, ys.ctypes.data, yst.ctypes.data,
                                       len(X), C.byref(p), res.ctypes.data, paths.ctypes.data, cap,
                                       C.byref(used), C.byref(ms))
        if rc:
            raise ImsameError(rc, "imsame_dev_nw_pairs")
        return res, paths[:used.value], ms.value

    def revcomp(self, data):
        """reverseComplement.c on the device: FASTA bytes -> FASTA bytes."""
        src = np.frombuffer(data, dtype=np.uint8)
        cap = len(data) + data.count(b">") + 2
        while True:
            out = np.zeros(max(cap, 1), dtype=np.uint8)
            ol = C.c_uint64()
            rc = lib().imsame_dev_revcomp(self._h, src.ctypes.data if len(src) else None, len(src),
                                          out.ctypes.data, cap, C.byref(ol))
            if rc == abi.IMSAME_E_ARG and ol.value > cap:
                cap = ol.value
                continue
            if rc:
                raise ImsameError(rc, "imsame_dev_revcomp")
            return out[:ol.value].tobytes()
