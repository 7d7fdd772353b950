"""CPU tests of the host I/O contracts (csrc/vame_io.cpp through libvame.so):
frame ingest vs the reference's reader semantics, and the decision-log writer
byte-for-byte vs the restatement of reportAffineResultsMaster_new
(tests/oracle_log.py), fed with the reference kernels' own outputs
(tests/golden/*.npz).  Also the CLI's argument handling (no GPU needed)."""
import glob
import os
import subprocess

import numpy as np
import pytest

from vame import logs
from vame.synth import synth_sequence, write_csv

import oracle_log as OL

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = sorted(glob.glob(os.path.join(REPO, "tests", "golden", "s*_*.npz")))  # pair fixtures (s416_*, s832_*)
CLI = os.path.join(REPO, "vvc-affine-gpu_amd", "bin", "vame")
MODES = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")


# ------------------------------------------------------------------ ingest
@pytest.fixture(scope="module")
def seq416():
    return synth_sequence(416, 240, 3, qp=32)


@pytest.mark.parametrize("nthreads", [1, 3, 8])
def test_read_csv_matches_writer(tmp_path, seq416, nthreads):
    orig, recon = seq416
    p = str(tmp_path / "orig.csv")
    write_csv(p, orig)
    got = logs.read_frames(p, 416, 240, 3, nthreads)
    assert got.dtype == np.uint16 and (got == orig).all()
    # fewer frames than the file holds: only the first ones are read
    assert (logs.read_frames(p, 416, 240, 2, nthreads) == orig[:2]).all()


def test_read_csv_reference_semantics(tmp_path):
    """getline(',') + stoi per value: leading blanks, trailing commas, CRLF,
    '+' signs, text after the digits, extra columns, no final newline."""
    rng = np.random.default_rng(7)
    fr = rng.integers(0, 1024, size=(2, 240, 416)).astype(np.uint16)
    lines = []
    for k in range(2):
        for h in range(240):
            v = [str(x) for x in fr[k, h]]
            if h % 5 == 1:
                v = [" " + s for s in v]
            if h % 7 == 2:
                v[0] = v[0].replace(v[0].strip(), "+" + v[0].strip())
            if h % 11 == 3:
                v[3] = v[3] + "abc"
            line = ",".join(v)
            if h % 3 == 0:
                line += ","
            if h % 4 == 0:
                line += ",99,98"  # extra columns are ignored
            if h % 6 == 5:
                line += "\r"
            lines.append(line)
    p = tmp_path / "odd.csv"
    p.write_text("\n".join(lines))  # no trailing newline
    got = logs.read_frames(str(p), 416, 240, 2, 4)
    assert (got == fr).all()
    assert (OL.read_frames(str(p), 416, 240, 2) == fr).all()


def test_read_frames_errors_and_raw(tmp_path):
    rng = np.random.default_rng(3)
    fr = rng.integers(0, 1024, size=(1, 240, 416)).astype(np.uint16)
    p = str(tmp_path / "one.csv")
    write_csv(p, fr)
    with pytest.raises(Exception):
        logs.read_frames(p, 416, 240, 2)  # short file
    with pytest.raises(Exception):
        logs.read_frames(str(tmp_path / "missing.csv"), 416, 240, 1)
    bad = tmp_path / "bad.csv"
    bad.write_text("1,2,x3\n" * 240)
    with pytest.raises(Exception):
        logs.read_frames(str(bad), 3, 240, 1)
    short = tmp_path / "short.csv"
    short.write_text("1,2\n" * 240)
    with pytest.raises(Exception):
        logs.read_frames(str(short), 3, 240, 1)
    # stoi's out_of_range: a value beyond int's range is rejected, not wrapped
    for big in ("2147483648", "-2147483649", "99999999999999999999999"):
        over = tmp_path / "over.csv"
        over.write_text(f"1,{big},3\n" * 240)
        with pytest.raises(Exception):
            logs.read_frames(str(over), 3, 240, 1)
    edge = tmp_path / "edge.csv"  # int's own limits are accepted (stored as unsigned short)
    edge.write_text("2147483647,-2147483648,65537\n" * 240)
    got = logs.read_frames(str(edge), 3, 240, 1)
    assert (got[0, :, 0] == 0xFFFF).all() and (got[0, :, 1] == 0).all() and (got[0, :, 2] == 1).all()
    raw = str(tmp_path / "f.u16")
    fr.tofile(raw)
    assert (logs.read_frames(raw, 416, 240, 1) == fr).all()


def test_read_csv_large_multithreaded(tmp_path):
    """Many byte ranges, lines straddling range cuts: 832x480, 2 frames, 16 threads."""
    rng = np.random.default_rng(11)
    fr = rng.integers(0, 1024, size=(2, 480, 832)).astype(np.uint16)
    p = str(tmp_path / "big.csv")
    write_csv(p, fr)
    for t in (2, 7, 16, 64):
        assert (logs.read_frames(p, 832, 480, 2, t) == fr).all()


# ------------------------------------------------------------------ decision log
def _files(d):
    return sorted(os.listdir(d))


def _golden_results(z):
    return {m: (z[m + "_cost"], np.concatenate([np.full((len(z[m + "_cost"]), 1), 2 + (i & 1),
                                                        np.int32), z[m + "_cpmv"]], 1))
            for i, m in enumerate(MODES)}


@pytest.mark.parametrize("path", GOLDEN[:4], ids=[os.path.basename(p)[:-4] for p in GOLDEN[:4]])
def test_log_writer_byte_identical(tmp_path, path):
    z = np.load(path)
    W, H = int(z["W"]), int(z["H"])
    res = _golden_results(z)
    a, b = tmp_path / "native", tmp_path / "restated"
    a.mkdir()
    b.mkdir()
    # two (POC, ref) appends after the headers, like POC 1 ref 0 then POC 2 ref 1
    for pred, m in enumerate(MODES):
        cost, cp = res[m]
        logs.write_headers(str(a / "log"), pred)
        OL.write_headers(str(b / "log"), pred)
        for poc, ref in ((1, 0), (2, 1)):
            nb = logs.append(str(a / "log"), pred, W, H, poc, ref, cost, cp, nthreads=3)
            assert nb > 0
            OL.append(str(b / "log"), pred, W, H, poc, ref, cost, cp)
    fa, fb = _files(a), _files(b)
    assert fa == fb
    assert len(fa) == 40  # 12 FULL + 8 HALF names, x {2, 3} CPs
    for f in fa:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f
    # row count: every candidate CU of every CTU, twice
    n_ctus = logs.lib().vame_num_ctus(W, H)
    for pred in range(4):
        rows = sum(len((a / f).read_text().splitlines()) - 1
                   for f in fa if OL.TYPES[pred] in "_" + f[4:])
        assert rows == 2 * n_ctus * (284 if pred >= 2 else 201)


def test_log_counts_and_remove_old(tmp_path):
    assert [logs.lib().vame_log_file_count(p) for p in range(4)] == [12, 12, 8, 8]
    pre = str(tmp_path / "x")
    for pred in range(4):
        logs.write_headers(pre, pred)
    assert len(_files(tmp_path)) == 40
    (tmp_path / "keep.csv").write_text("k")
    logs.remove_old(pre)
    assert _files(tmp_path) == ["keep.csv"]
    # the restated removeOldTraces covers the same names
    for pred in range(4):
        OL.write_headers(pre, pred)
    OL.remove_old(pre)
    assert _files(tmp_path) == ["keep.csv"]


def test_write_poc_order(tmp_path):
    """write_poc == the reference's per-POC sequence (refIdx outer, PRED inner)."""
    z = np.load(GOLDEN[0])
    W, H = int(z["W"]), int(z["H"])
    res = _golden_results(z)
    results = {(r, m): res[m] for r in range(2) for m in MODES}
    a, b = tmp_path / "a", tmp_path / "b"
    a.mkdir()
    b.mkdir()
    for poc in (1, 2):
        logs.write_poc(str(a / "p"), W, H, poc, results, nthreads=2)
        for r in range(2):
            for pred, m in enumerate(MODES):
                if poc == 1 and r == 0:
                    OL.write_headers(str(b / "p"), pred)
                OL.append(str(b / "p"), pred, W, H, poc, r, *res[m])
    for f in _files(a):
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def test_log_tables_equal_kernel_geometry():
    """The host tables the reference's writer indexes (constants.h) are the
    kernel's CU geometry (constants.cl) restated in vame_tables.h."""
    from vame.hostlogic import geometry
    for align, key in ((0, "full"), (1, "half")):
        geo = geometry(align)
        for g, t in enumerate(OL.TABLES[key]):
            w, h, xs, ys, stride = geo[g]
            assert (w, h, len(xs), stride) == (t["w"], t["h"], t["n"], t["stride"]), (key, g)
            if align:
                assert list(xs) == t["x"] and list(ys) == t["y"], g
            else:
                k = np.arange(t["n"])
                assert list(xs) == list((k * w) % 128) and list(ys) == list((k * w) // 128 * h)


# ------------------------------------------------------------------ CLI (no GPU)
def _run(args, cwd):
    return subprocess.run([CLI] + args, cwd=cwd, capture_output=True, text=True, timeout=60)


def test_cli_help_and_parameter_errors(tmp_path):
    r = _run(["--help"], tmp_path)
    assert r.returncode == 1 and "--FramesToBeEncoded" in r.stdout and "-q [ --QP ]" in r.stdout
    r = _run(["-q", "32"], tmp_path)
    assert r.returncode == 1
    for msg in ("QP=32", "[!] ERROR: FramesToBeEncoded not set.", "[!] ERROR: Resolution not set.",
                "[!] ERROR: Input original frames not set.",
                "Exiting after finding errors in input parameters"):
        assert msg in r.stdout, msg
    r = _run(["--bogus", "1"], tmp_path)
    assert r.returncode == 1 and "unrecognised option" in r.stderr
    r = _run(["-q", "32", "-f", "1", "-s", "416x240", "-o", "a", "-r", "b", "--align", "diag"], tmp_path)
    assert r.returncode == 1 and "--align must be both, full or half" in r.stdout
    # boost-style forms: -q32, --QP=32, unique long prefix (--Frames), defaults reported
    r = _run(["-q32", "--Frames=3", "--Res", "416x240", "-o", "a", "-r", "b",
              "--ExtraGradientIter", "2"], tmp_path)
    for msg in ("QP=32", "FramesToBeEncoded=3", "Resolution=416x240", "InputOriginalFrame=a",
                "ExtraGradientIter=2. Using a total of 7 iterations for 2 CPs and 6 iterations",
                "Device index not set. Using standard value of 0.",
                "CPMVs log file not set."):
        assert msg in r.stdout, msg


def test_cli_no_device_or_bad_resolution(tmp_path):
    """Without a HIP device the CLI stops like the reference with a bad index."""
    r = _run(["-q", "32", "-f", "1", "-s", "416x240", "-o", "a", "-r", "b"], tmp_path)
    if "Incorrect GPU index" in r.stdout:
        assert r.returncode == 0
    else:  # a GPU is present: then the inputs are missing
        assert r.returncode == 1 and "error while opening samples files" in r.stderr


@pytest.mark.parametrize("size,nrefs,mask", [((416, 240), 2, 15), ((1920, 1080), 4, 15),
                                             ((1280, 720), 3, 5)])
def test_log_writer_poc_equals_appends(tmp_path, size, nrefs, mask):
    """vame_log_writer_poc (a whole POC per call, persistent pool, files kept
    open) writes the bytes of the reference-order per-(POC, refIdx, PRED)
    appends, including the HALF names shared by several groups."""
    W, H = size
    rng = np.random.default_rng(W + nrefs)
    n_ctus = logs.lib().vame_num_ctus(W, H)
    preds = [m for m in range(4) if (mask >> m) & 1]
    a, b = tmp_path / "writer", tmp_path / "appends"
    a.mkdir()
    b.mkdir()
    with logs.LogWriter(str(a / "log"), W, H, nthreads=5) as wr:
        for poc in (1, 2, 3):
            res = {}
            for r in range(min(nrefs, poc)):
                for m in preds:
                    n = n_ctus * (284 if m >> 1 else 201)
                    cp = rng.integers(-70000, 70000, (n, 7)).astype(np.int32)
                    res[(r, logs.PREDS[m])] = (rng.integers(0, 1 << 40, n), cp)
            nb = logs.write_poc(str(a / "log"), W, H, poc, res, writer=wr)
            nb2 = logs.write_poc(str(b / "log"), W, H, poc, res, nthreads=3)
            assert nb == nb2 > 0
    fa, fb = _files(a), _files(b)
    assert fa == fb and len(fa) == sum(logs.lib().vame_log_file_count(m) for m in preds)
    for f in fa:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f


def test_log_writer_rejects_bad_arguments(tmp_path):
    import ctypes
    L = logs.lib()
    assert not L.vame_log_writer_create(str(tmp_path / "x").encode(), 1000, 1000, 1)
    w = L.vame_log_writer_create(str(tmp_path / "x").encode(), 416, 240, 1)
    assert w
    nul = (ctypes.c_void_p * 4)()
    assert L.vame_log_writer_poc(w, 1, 1, 1, nul, nul) < 0  # PRED 0 in the mask without arrays
    assert L.vame_log_writer_poc(w, 1, 5, 1, nul, nul) < 0  # more than 4 refs
    assert L.vame_log_writer_destroy(w) == 0


def test_pred_mask_mirrors_the_abi():
    """vame.engine.pred_mask == the library's vame_pred_mask for every valid
    mode mask: 2-CP [+ 3-CP] per alignment, both alignments unless one is selected."""
    from vame.engine import pred_mask
    masks = (1, 3, 5, 7, 9, 11, 13, 15)
    assert [pred_mask(m) for m in masks] == [5, 15, 1, 3, 4, 12, 5, 15]
    assert [logs.lib().vame_pred_mask(m) for m in masks] == [pred_mask(m) for m in masks]


def _random_poc(rng, W, H, refs, preds=range(4)):
    n_ctus = logs.lib().vame_num_ctus(W, H)
    res = {}
    for r in refs:
        for m in preds:
            n = n_ctus * (284 if m >> 1 else 201)
            res[(r, logs.PREDS[m])] = (rng.integers(0, 1 << 31, n),
                                       rng.integers(-70000, 70000, (n, 7)).astype(np.int32))
    return res


def test_log_append_concurrent_threads(tmp_path):
    """vame_log_append from two threads at once (ctypes drops the GIL): each
    call runs its own threads, so both logs equal a serial run."""
    import threading
    rng = np.random.default_rng(5)
    res = [_random_poc(rng, 1920, 1080, [0]) for _ in range(2)]
    def job(k, d, reps):
        for _ in range(reps):
            for m, name in enumerate(logs.PREDS):
                logs.append(str(d / f"log{k}"), m, 1920, 1080, 1, 0, *res[k][(0, name)], nthreads=4)
    par, ser = tmp_path / "par", tmp_path / "ser"
    par.mkdir()
    ser.mkdir()
    th = [threading.Thread(target=job, args=(k, par, 3)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(2):
        job(k, ser, 3)
    fa = _files(par)
    assert fa == _files(ser) and len(fa) == 80
    for f in fa:
        assert (par / f).read_bytes() == (ser / f).read_bytes(), f


def test_log_writer_refs_and_fork(tmp_path):
    """vame_log_writer_refs (a POC's refIdx range cut between frame-shard
    ranks): the two halves written one after the other equal the whole POC;
    and a writer whose pool started before a fork() still works in the child
    (serially) instead of waiting for threads the child does not have."""
    rng = np.random.default_rng(8)
    res = _random_poc(rng, 416, 240, range(4))
    a, b = tmp_path / "whole", tmp_path / "halves"
    a.mkdir()
    b.mkdir()
    with logs.LogWriter(str(a / "log"), 416, 240, nthreads=3) as w:
        w.poc(7, res)
    with logs.LogWriter(str(b / "log"), 416, 240, nthreads=3) as w:
        w.poc(7, {k: v for k, v in res.items() if k[0] < 1})
        w.poc(7, {k: v for k, v in res.items() if k[0] >= 1})
    for f in _files(a):
        assert (a / f).read_bytes() == (b / f).read_bytes(), f
    with pytest.raises(ValueError):
        logs.LogWriter(str(b / "bad"), 416, 240).poc(7, {k: v for k, v in res.items() if k[0] != 1})
    c = tmp_path / "forked"
    c.mkdir()
    w = logs.LogWriter(str(c / "log"), 416, 240, nthreads=4)
    w.poc(7, {k: v for k, v in res.items() if k[0] < 1})  # pool threads are running now
    pid = os.fork()
    if pid == 0:  # child: finish the POC with the inherited writer, then leave at once
        try:
            w.poc(7, {k: v for k, v in res.items() if k[0] >= 1})
            w.close()
            os._exit(0)
        except BaseException:
            os._exit(1)
    _, status = os.waitpid(pid, 0)
    assert os.waitstatus_to_exitcode(status) == 0
    for f in _files(a):
        assert (a / f).read_bytes() == (c / f).read_bytes(), f
    w._w = None  # the parent's copy: its files were completed by the child


def test_read_frames_range(tmp_path):
    """vame_read_frames_range: frames first .. first+n-1 of a CSV / raw file
    (a frame-sharded rank's share), equal to the slice of a whole read."""
    rng = np.random.default_rng(3)
    fr = rng.integers(0, 1024, size=(5, 240, 416)).astype(np.uint16)
    p = str(tmp_path / "f.csv")
    write_csv(p, fr)
    fr.tofile(str(tmp_path / "f.u16"))
    for path in (p, str(tmp_path / "f.u16")):
        for first, n in ((0, 5), (2, 3), (4, 1), (1, 2)):
            for t in (1, 5):
                assert (logs.read_frames(path, 416, 240, n, t, first=first) == fr[first:first + n]).all()
        with pytest.raises(logs.VameError):
            logs.read_frames(path, 416, 240, 2, first=4)


@pytest.mark.parametrize("K", [1, 3, 7, 40])
def test_read_frames_span_from_chunk_index(tmp_path, K):
    """vame_count_lines over K byte chunks + line_span + vame_read_frames_span
    (the frame-shard ranks' ingest): any frame range read through the chunks
    that hold it equals the slice of a whole read; the bytes ahead of the span
    are never parsed."""
    rng = np.random.default_rng(K)
    fr = rng.integers(0, 1024, size=(6, 240, 416)).astype(np.uint16)
    p = str(tmp_path / "f.csv")
    write_csv(p, fr)
    size = os.path.getsize(p)
    bounds = [size * k // K for k in range(K + 1)]
    counts = [logs.count_lines(p, bounds[k], bounds[k + 1], nthreads=3) for k in range(K)]
    assert sum(counts) == logs.count_lines(p) == 6 * 240
    # the batched form: every chunk at once, any subset, empty ranges, any order
    assert logs.count_lines_ranges(p, [(bounds[k], bounds[k + 1]) for k in range(K)], nthreads=3) == counts
    sub = list(range(K - 1, -1, -2))
    assert logs.count_lines_ranges(p, [(bounds[k], bounds[k + 1]) for k in sub]) == [counts[k] for k in sub]
    assert logs.count_lines_ranges(p, [(5, 5), (0, size), (size, size + 10)]) == [0, 6 * 240, 0]
    assert logs.count_lines_ranges(p, []) == []
    with pytest.raises(logs.VameError):
        logs.count_lines_ranges(p, [(10, 5)])
    prefix = [0] + list(np.cumsum(counts))
    for first, n in ((0, 6), (0, 1), (2, 3), (5, 1), (3, 2)):
        span = logs.line_span(bounds, prefix, first * 240, (first + n) * 240)
        assert span[0] <= size and span[2] <= size
        got = logs.read_frames(p, 416, 240, n, 4, first=first, span=span)
        assert (got == fr[first:first + n]).all(), (first, n, span)
    # a span that misses the frames' last line is refused
    with pytest.raises(logs.VameError):
        logs.read_frames(p, 416, 240, 3, first=0, span=(0, 0, size // 3))


def test_log_writer_deferred_flush_at(tmp_path):
    """Deferred writers (vame_log_writer_set_deferred / _sizes / _flush_at):
    three writers each hold one block of POCs (one block starts inside POC 5,
    at refIdx 2) and place it into the same files at the byte offsets of the
    blocks before it; the files equal one writer appending every POC."""
    rng = np.random.default_rng(12)
    pocs = {p: _random_poc(rng, 416, 240, range(min(4, p))) for p in range(1, 8)}
    a = tmp_path / "one"
    a.mkdir()
    with logs.LogWriter(str(a / "log"), 416, 240) as w:
        for p, res in pocs.items():
            logs.write_poc(str(a / "log"), 416, 240, p, res, writer=w)
    b = tmp_path / "three"
    b.mkdir()
    pre = str(b / "log")
    cut = {k: v for k, v in pocs[5].items() if k[0] < 2}, {k: v for k, v in pocs[5].items() if k[0] >= 2}
    blocks = [[(p, pocs[p]) for p in (1, 2, 3)], [(4, pocs[4]), (5, cut[0])], [(5, cut[1]), (6, pocs[6]), (7, pocs[7])]]
    writers = [logs.LogWriter(pre, 416, 240, nthreads=3) for _ in blocks]
    for k in (1, 2):
        writers[k].defer()
    for w, blk in zip(writers, blocks):
        for p, res in blk:
            logs.write_poc(pre, 416, 240, p, res, writer=w)
    writers[0].close()
    with pytest.raises(logs.VameError):  # the mode is fixed once rows were logged
        writers[1].defer()
    names = writers[1].files()
    assert names == logs.log_names(pre)
    base = [os.path.getsize(n) if os.path.exists(n) else 0 for n in names]
    s1, s2 = writers[1].held_sizes(), writers[2].held_sizes()
    # flush the later block first: the files grow with holes, then fill in
    writers[2].flush_at([x + y for x, y in zip(base, s1)])
    writers[1].flush_at(base)
    for w in writers[1:]:
        w.close()
    fa = _files(a)
    assert fa == _files(b) and len(fa) == 40
    for f in fa:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f
