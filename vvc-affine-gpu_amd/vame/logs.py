"""Host I/O contracts of the reference's ./main, through libvame.so:
frame ingest (main.cpp:293-330) and the per-CU decision log
(main_aux_functions.h:387-525, 1547-1585).  Native and multi-threaded
(csrc/vame_io.cpp); these are thin numpy wrappers."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import VameError, lib

PREDS = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")  # constants.h:15-21 PRED_TYPES
CPMVS_DTYPE = np.dtype([("nCPs", "<i4"), ("LTx", "<i4"), ("LTy", "<i4"), ("RTx", "<i4"),
                        ("RTy", "<i4"), ("LBx", "<i4"), ("LBy", "<i4")])


def read_frames(path: str, width: int, height: int, n_frames: int, nthreads: int = 0,
                first: int = 0, span=None) -> np.ndarray:
    """(n_frames, H, W) uint16 from a reference-layout CSV (or raw .u16/.yuv):
    frames first .. first + n_frames - 1 of the file.  span = (begin,
    lines_before, end): only bytes [begin, end) are read (see line_span)."""
    out = np.empty((n_frames, height, width), np.uint16)
    b, lb, e = span if span is not None else (0, 0, -1)
    rc = lib().vame_read_frames_span(path.encode(), width, height, first, n_frames, b, lb, e,
                                     out.ctypes.data_as(ctypes.c_void_p), nthreads)
    if rc != 0:
        raise VameError(f"cannot read frames {first}..{first + n_frames - 1} of {width}x{height} "
                        f"from {path} (rc={rc})")
    return out


def count_lines(path: str, begin: int = 0, end: int = -1, nthreads: int = 0) -> int:
    """Number of '\\n' in bytes [begin, end) of a file (end < 0: to the end)."""
    n = lib().vame_count_lines(path.encode(), begin, end, nthreads)
    if n < 0:
        raise VameError(f"cannot read {path}")
    return n


def count_lines_ranges(path: str, ranges, nthreads: int = 0) -> list[int]:
    """'\\n' counts of several byte ranges [(begin, end), ...] of one file,
    in one native pass (vame_count_lines_ranges)."""
    b = np.ascontiguousarray([r[0] for r in ranges], dtype=np.int64)
    e = np.ascontiguousarray([r[1] for r in ranges], dtype=np.int64)
    out = np.zeros(len(ranges), dtype=np.int64)
    rc = lib().vame_count_lines_ranges(path.encode(), b.ctypes.data_as(ctypes.c_void_p),
                                       e.ctypes.data_as(ctypes.c_void_p), len(ranges),
                                       out.ctypes.data_as(ctypes.c_void_p), nthreads)
    if rc != 0:
        raise VameError(f"cannot count the lines of {path} (rc={rc})")
    return out.tolist()


def line_span(bounds: list[int], prefix: list[int], line0: int, line1: int) -> tuple[int, int, int]:
    """(begin, lines_before, end) of the chunks that hold text lines [line0,
    line1), from chunk byte bounds[0..K] and prefix[k] = the newlines ahead of
    bounds[k] (line L starts after newline L - 1)."""
    import bisect
    K = len(bounds) - 1
    if line0 == 0:
        b, lb = 0, 0
    else:
        k0 = min(bisect.bisect_right(prefix, line0 - 1) - 1, K - 1)
        b, lb = bounds[k0], prefix[k0]
    k1 = bisect.bisect_right(prefix, line1 - 1) - 1  # chunk of the last line's newline
    return b, lb, bounds[min(k1 + 1, K)]


def log_names(prefix: str, pred_mask: int = 15) -> list[str]:
    """The distinct decision-log files of the PREDs in pred_mask, in PRED and
    group order (main_aux_functions.h:392-425: HALF groups of one W x H share a file)."""
    names = []
    L = lib()
    w, h, n, st = (ctypes.c_int() for _ in range(4))
    xs, ys = (ctypes.c_int * 64)(), (ctypes.c_int * 64)()
    for m, tag in enumerate(PREDS):
        if not (pred_mask >> m) & 1:
            continue
        for g in range(L.vame_num_groups(m >> 1)):
            L.vame_group_geometry(m >> 1, g, ctypes.byref(w), ctypes.byref(h), ctypes.byref(n),
                                  ctypes.byref(st), xs, ys)
            name = f"{prefix}_{tag[:4]}_{tag[5]}CPs_{w.value}x{h.value}.csv"
            if name not in names:
                names.append(name)
    return names


def part_prefix(prefix: str, rank: int) -> str:
    """The prefix of rank `rank`'s part files (vame.distrun --shard-logs)."""
    return f"{prefix}.part{rank}"


def merge_parts(prefix: str, n_parts: int, pred_mask: int = 15) -> int:
    """Append the part files of ranks 1..n_parts-1 (headerless, in rank order)
    to rank 0's final files and remove them: the `cat` of the parts, byte for
    byte the one-process logs.  In-kernel copies at explicit offsets
    (os.copy_file_range; an O_APPEND descriptor would refuse them), plain
    pread / pwrite where the file system has none.  Returns the bytes appended."""
    finals = log_names(prefix, pred_mask)
    parts = [log_names(part_prefix(prefix, r), pred_mask) for r in range(1, n_parts)]
    moved = 0
    for i, name in enumerate(finals):
        dst = os.open(name, os.O_WRONLY | os.O_CREAT, 0o644)
        try:
            pos = os.fstat(dst).st_size
            for names in parts:
                if not os.path.exists(names[i]):
                    continue
                src = os.open(names[i], os.O_RDONLY)
                try:
                    size, off = os.fstat(src).st_size, 0
                    try:
                        while off < size:
                            n = os.copy_file_range(src, dst, size - off, off, pos + off)
                            if n <= 0:
                                break
                            off += n
                    except OSError:  # no in-kernel copy between these files
                        pass
                    while off < size:
                        buf = os.pread(src, min(16 << 20, size - off), off)
                        if not buf:
                            raise VameError(f"short read from {names[i]}")
                        off += os.pwrite(dst, buf, pos + off)
                finally:
                    os.close(src)
                pos += size
                moved += size
                os.remove(names[i])
        finally:
            os.close(dst)
    return moved


def remove_old(prefix: str) -> None:
    lib().vame_log_remove_old(prefix.encode())


def write_headers(prefix: str, pred: int) -> None:
    if lib().vame_log_write_headers(prefix.encode(), pred) != 0:
        raise VameError(f"cannot create log files {prefix}_*")


def append(prefix: str, pred: int, width: int, height: int, poc: int, ref: int,
           cost: np.ndarray, cpmvs: np.ndarray, nthreads: int = 0) -> int:
    """Rows of one (POC, refIdx, pred); cost int64[n], cpmvs = [n, 7] int32 or CPMVS_DTYPE[n]."""
    cost, cpmvs = _arrays(pred, width, height, cost, cpmvs)
    nb = lib().vame_log_append(prefix.encode(), pred, width, height, poc, ref,
                               cost.ctypes.data_as(ctypes.c_void_p),
                               cpmvs.ctypes.data_as(ctypes.c_void_p), nthreads)
    if nb < 0:
        raise VameError(f"writing log files {prefix}_* failed")
    return nb


def _arrays(pred: int, width: int, height: int, cost: np.ndarray, cpmvs: np.ndarray):
    cost = np.ascontiguousarray(cost, np.int64)
    cpmvs = np.ascontiguousarray(cpmvs)
    if cpmvs.dtype != CPMVS_DTYPE:
        cpmvs = np.ascontiguousarray(cpmvs, np.int32)
        assert cpmvs.ndim == 2 and cpmvs.shape[1] == 7
    n = lib().vame_num_ctus(width, height) * (284 if pred >> 1 else 201)
    if cost.shape[0] != n or cpmvs.shape[0] != n:
        raise ValueError(f"results must hold {n} entries")
    return cost, cpmvs


class LogWriter:
    """vame_log_writer: a whole POC per call on a persistent thread pool, files
    kept open; the bytes of the reference's per-(POC, refIdx, PRED) appends."""

    def __init__(self, prefix: str, width: int, height: int, nthreads: int = 0):
        self.width, self.height = width, height
        self._w = lib().vame_log_writer_create(prefix.encode(), width, height, nthreads)
        if not self._w:
            raise VameError(f"cannot create a log writer for {prefix} ({width}x{height})")

    def poc(self, poc: int, results) -> int:
        """results: {(ref, PRED name): (cost, cpmvs)}; refs r0..r0+n-1 (r0 = 0
        unless the POC is cut between frame-shard ranks), each with the same
        PREDs."""
        refs = sorted({r for r, _ in results})
        if not refs or refs != list(range(refs[0], refs[0] + len(refs))) or refs[-1] > 3:
            raise ValueError("refIdx must be a contiguous range within 0..3")
        r0 = refs[0]
        mask = 0
        for m, name in enumerate(PREDS):
            if any((r, name) in results for r in refs):
                mask |= 1 << m
        keep = []
        cost_p = (ctypes.c_void_p * (4 * len(refs)))()
        cp_p = (ctypes.c_void_p * (4 * len(refs)))()
        for r in refs:
            for m, name in enumerate(PREDS):
                if not (mask >> m) & 1:
                    continue
                if (r, name) not in results:
                    raise ValueError(f"refIdx {r} lacks {name}")
                c, p = _arrays(m, self.width, self.height, *results[(r, name)])
                keep += [c, p]
                cost_p[(r - r0) * 4 + m] = c.ctypes.data
                cp_p[(r - r0) * 4 + m] = p.ctypes.data
        nb = lib().vame_log_writer_refs(self._w, poc, r0, len(refs), mask, cost_p, cp_p)
        if nb < 0:
            raise VameError("writing the log files failed")
        return nb

    def defer(self) -> None:
        """Keep the rows in memory (vame_log_writer_set_deferred) until flush_at."""
        if lib().vame_log_writer_set_deferred(self._w, 1) != 0:
            raise VameError("vame_log_writer_set_deferred failed")

    def files(self) -> list[str]:
        """The writer's files, in its numbering."""
        L = lib()
        buf = ctypes.create_string_buffer(4096)
        out = []
        for f in range(L.vame_log_writer_num_files(self._w)):
            if L.vame_log_writer_file_name(self._w, f, buf, len(buf)) != 0:
                raise VameError("vame_log_writer_file_name failed")
            out.append(buf.value.decode())
        return out

    def held_sizes(self) -> list[int]:
        n = lib().vame_log_writer_num_files(self._w)
        arr = (ctypes.c_longlong * n)()
        lib().vame_log_writer_sizes(self._w, arr)
        return list(arr)

    def flush_at(self, offsets: list[int]) -> int:
        """Write every file's held rows at offsets[f] (vame_log_writer_flush_at)."""
        arr = (ctypes.c_longlong * len(offsets))(*offsets)
        nb = lib().vame_log_writer_flush_at(self._w, arr)
        if nb < 0:
            raise VameError("vame_log_writer_flush_at failed")
        return nb

    def close(self) -> None:
        if self._w:
            lib().vame_log_writer_destroy(self._w)
            self._w = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_poc(prefix: str, width: int, height: int, poc: int, results, nthreads: int = 0,
              writer: LogWriter | None = None) -> int:
    """Log one POC like main.cpp:942-958: for each refIdx the four PREDs in
    order (headers first at POC 1 / refIdx 0).  results: {(ref, PRED name):
    (cost, cpmvs)} as host arrays.  With a LogWriter (same prefix) the POC
    goes through it in one call."""
    refs = sorted({r for r, _ in results})
    if poc == 1 and 0 in refs:
        for m, name in enumerate(PREDS):
            if (0, name) in results:
                write_headers(prefix, m)
    if writer is not None:
        return writer.poc(poc, results)
    nb = 0
    for r in refs:
        for m, name in enumerate(PREDS):
            if (r, name) not in results:
                continue
            cost, cp = results[(r, name)]
            nb += append(prefix, m, width, height, poc, r, cost, cp, nthreads)
    return nb


if __name__ == "__main__":  # python -m vame.logs merge <prefix> <ranks> [all|2cp]
    import sys
    if len(sys.argv) not in (4, 5) or sys.argv[1] != "merge":
        sys.exit("usage: python -m vame.logs merge <log prefix> <ranks> [all|2cp]")
    mask = 5 if len(sys.argv) == 5 and sys.argv[4] == "2cp" else 15
    print(f"{merge_parts(sys.argv[2], int(sys.argv[3]), mask)} bytes appended")
