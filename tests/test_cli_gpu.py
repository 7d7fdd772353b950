"""End-to-end drop-in check of the `vame` CLI on MI355X: CSV frames in, the 40
per-CU decision-log CSVs out, byte-identical to the reference's log writer
(restated in tests/oracle_log.py from main_aux_functions.h:387-525) applied to
the CPU oracle's results for every (POC, refIdx) the reference host visits
(ring of main.cpp:591-707, lambda of main.cpp:585)."""
import os
import subprocess

import numpy as np
import pytest

from vame.hostlogic import lambda_for_poc, ref_list
from vame.synth import synth_sequence, write_csv

import oracle_log as OL
import oracle_py as O

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "vvc-affine-gpu_amd", "bin", "vame")
PREDS = {(0, 2): 0, (0, 3): 1, (1, 2): 2, (1, 3): 3}


def expected_logs(d, orig, recon, qp, extra=0, modes=(2, 3), prof=False):
    """Oracle results -> restated writer, in the reference host's order."""
    n, H, W = orig.shape
    pre = str(d / "log")
    for poc in range(1, n + 1):
        lam = lambda_for_poc(qp, poc)
        for r, label in enumerate(ref_list(poc)):
            res = O.affine_me_pair(recon[label], orig[poc - 1], lam, extra=extra, modes=modes,
                                   prof=prof)
            for (align, ncp), pred in sorted(PREDS.items(), key=lambda kv: kv[1]):
                if (align, ncp) not in res:
                    continue
                if poc == 1 and r == 0:
                    OL.write_headers(pre, pred)
                cost, cp = res[(align, ncp)]
                cp7 = np.stack([cp[f] for f in ("nCPs", "LTx", "LTy", "RTx", "RTy", "LBx", "LBy")],
                               1)
                OL.append(pre, pred, W, H, poc, r, cost, cp7)


def run_cli(tmp, W, H, n, qp, extra_args=(), name="out"):
    out = tmp / name
    out.mkdir()
    args = [CLI, "-f", str(n), "-s", f"{W}x{H}", "-q", str(qp), "-o", str(tmp / "orig.csv"),
            "-r", str(tmp / "recon.csv"), "-l", str(out / "log"), *extra_args]
    r = subprocess.run(args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return out, r.stdout


def compare_dirs(a, b):
    fa, fb = sorted(os.listdir(a)), sorted(os.listdir(b))
    assert fa == fb
    for f in fa:
        assert (a / f).read_bytes() == (b / f).read_bytes(), f
    return fa


@pytest.fixture(scope="module")
def seq416(tmp_path_factory):
    tmp = tmp_path_factory.mktemp("s416")
    orig, recon = synth_sequence(416, 240, 6, qp=32)
    write_csv(str(tmp / "orig.csv"), orig)
    write_csv(str(tmp / "recon.csv"), recon)
    exp = tmp / "expected"
    exp.mkdir()
    expected_logs(exp, orig, recon, 32)
    return tmp, orig, recon, exp


def test_cli_logs_byte_identical_416(seq416):
    """6 POCs (1..4 refs, full ring), all four PREDs, fused per-POC launches."""
    tmp, orig, recon, exp = seq416
    out, stdout = run_cli(tmp, 416, 240, 6, 32)
    files = compare_dirs(out, exp)
    assert len(files) == 40
    # stdout keeps the reference's report order and keys
    lines = [l for l in stdout.splitlines() if "  RefIdx  " in l]
    assert lines[0].startswith("POC   1  RefIdx  0  -> lambda 78.949")
    assert len(lines) == 1 + 2 + 3 + 4 + 4 + 4
    assert stdout.count("Reporting results POC=") == 4 * len(lines)
    for key in ("TIMING RESULTS (nanoseconds)", "FULL_2CP_EXEC,", "TOTAL_EXEC_TIME(6x),",
                "OVERALL(6x),", "Writing headers", "FINISH HOST", "READ_CSV_TIME,", "LOG_WRITE_TIME,"):
        assert key in stdout, key
    # fused launches: the reference's per-PRED keys carry the fused kernel time
    # apportioned by algorithmic work -- all non-zero, summing to FUSED_POC_EXEC
    t = {l.split(",")[0]: float(l.split(",")[1]) for l in stdout.splitlines()
         if l.count(",") == 1 and l.split(",")[1].replace(".", "").isdigit()}
    preds = [t[k] for k in ("FULL_2CP_EXEC", "FULL_3CP_EXEC", "HALF_2CP_EXEC", "HALF_3CP_EXEC")]
    assert all(v > 0 for v in preds)
    assert abs(sum(preds) - t["FUSED_POC_EXEC"]) <= 1e-3 * t["FUSED_POC_EXEC"] + 4
    assert t["TOTAL_EXEC_TIME(6x)"] == t["FUSED_POC_EXEC"]
    assert preds[0] > preds[1] and preds[2] > preds[3]  # 6 vs 5 predictions per iteration set
    assert "PRED_EXEC_SOURCE,estimated-apportioned" in stdout.splitlines()  # named as estimates


def test_cli_per_launch_and_two_workers_identical(seq416):
    """The reference's launch pattern (4 launches per refIdx) and a 2-worker
    frame shard (two contexts on one GPU) give the same bytes."""
    tmp, orig, recon, exp = seq416
    out, stdout = run_cli(tmp, 416, 240, 6, 32, ["--per-launch"], name="per_launch")
    compare_dirs(out, exp)
    t = {l.split(",")[0]: float(l.split(",")[1]) for l in stdout.splitlines()
         if l.endswith(tuple("0123456789")) and "_EXEC," in l}
    assert all(t[k] > 0 for k in ("FULL_2CP_EXEC", "FULL_3CP_EXEC", "HALF_2CP_EXEC",
                                  "HALF_3CP_EXEC"))
    # per launch the keys are the launches' own event times, summing to TOTAL_EXEC_TIME
    assert "PRED_EXEC_SOURCE,measured" in stdout.splitlines()
    total = [float(l.split(",")[1]) for l in stdout.splitlines() if l.startswith("TOTAL_EXEC_TIME(")][0]
    assert abs(sum(t[k] for k in ("FULL_2CP_EXEC", "FULL_3CP_EXEC", "HALF_2CP_EXEC", "HALF_3CP_EXEC"))
               - total) <= 0.02 * total
    out2, _ = run_cli(tmp, 416, 240, 6, 32, ["--devices", "0,0", "--threads", "3"],
                      name="two_workers")
    compare_dirs(out2, exp)


def test_cli_three_workers_chunk_dealing(tmp_path):
    """--devices with 3 workers over 13 POCs: 4-POC chunks dealt in turn (POCs
    1-4, 5-8, 9-12 to workers 0, 1, 2 and POC 13 back to worker 0), fused and
    per-launch; the 40 logs equal the 1-worker run byte for byte."""
    orig, recon = synth_sequence(416, 240, 13, qp=27, seed=3)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    one, _ = run_cli(tmp_path, 416, 240, 13, 27, name="one")
    assert len(compare_dirs(run_cli(tmp_path, 416, 240, 13, 27, ["--devices", "0,0,0"],
                                    name="three")[0], one)) == 40
    compare_dirs(run_cli(tmp_path, 416, 240, 13, 27, ["--devices", "0,0,0", "--per-launch"],
                         name="three_pl")[0], one)


def test_cli_align_selection(seq416):
    """--align full / half (SURVEY §8f CLI extension): each run launches one
    alignment's items only and writes exactly that alignment's files, byte
    for byte the reference writer's; together they are the both-run."""
    tmp, orig, recon, exp = seq416
    seen = []
    for align in ("full", "half"):
        out, stdout = run_cli(tmp, 416, 240, 6, 32, ["--align", align], name=f"align_{align}")
        files = sorted(os.listdir(out))
        assert files and all(align.upper() in f for f in files), files
        for f in files:
            assert (out / f).read_bytes() == (exp / f).read_bytes(), f
        t = {l.split(",")[0]: float(l.split(",")[1]) for l in stdout.splitlines()
             if l.endswith(tuple("0123456789")) and "_EXEC," in l}
        other = "HALF" if align == "full" else "FULL"
        assert t[f"{other}_2CP_EXEC"] == 0 and t[f"{other}_3CP_EXEC"] == 0
        assert t[f"{align.upper()}_2CP_EXEC"] > 0 and t[f"{align.upper()}_3CP_EXEC"] > 0
        seen += files
    assert sorted(seen) == sorted(os.listdir(exp))


def test_cli_2cp_only_and_extra_iters(tmp_path):
    orig, recon = synth_sequence(416, 240, 3, qp=37, seed=0x1234)
    write_csv(str(tmp_path / "orig.csv"), orig)
    orig.tofile(str(tmp_path / "orig.u16"))
    recon.tofile(str(tmp_path / "recon.u16"))
    write_csv(str(tmp_path / "recon.csv"), recon)
    exp = tmp_path / "expected"
    exp.mkdir()
    expected_logs(exp, orig, recon, 37, extra=1, modes=(2,))
    out, _ = run_cli(tmp_path, 416, 240, 3, 37, ["--modes", "2cp", "--ExtraGradientIter", "1"])
    files = compare_dirs(out, exp)
    assert len(files) == 20
    # raw 16-bit inputs take the same path
    args = [CLI, "-f", "3", "-s", "416x240", "-q", "37", "-o", str(tmp_path / "orig.u16"),
            "-r", str(tmp_path / "recon.u16"), "-l", str(tmp_path / "raw_log"), "--modes", "2cp",
            "--ExtraGradientIter", "1"]
    assert subprocess.run(args, capture_output=True, timeout=300).returncode == 0
    for f in files:
        assert (tmp_path / ("raw_" + f)).read_bytes() == (exp / f).read_bytes()


def test_cli_1080p_c1(tmp_path):
    """BASELINE configs[0] shape: 1920x1080 QP32, 2 frames, all modes."""
    orig, recon = synth_sequence(1920, 1080, 2, qp=32)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    exp = tmp_path / "expected"
    exp.mkdir()
    expected_logs(exp, orig, recon, 32)
    out, _ = run_cli(tmp_path, 1920, 1080, 2, 32)
    files = compare_dirs(out, exp)
    assert len(files) == 40
    rows = sum(len((out / f).read_text().splitlines()) - 1 for f in files)
    assert rows == 3 * 130950  # 3 pairs x 130,950 rows (FULL + HALF, 2 + 3 CPs)


def test_cli_prof_416(tmp_path):
    """--prof: the logs equal the restated writer on the oracle's PROF results."""
    orig, recon = synth_sequence(416, 240, 3, qp=27, seed=0x50F)
    write_csv(str(tmp_path / "orig.csv"), orig)
    write_csv(str(tmp_path / "recon.csv"), recon)
    exp = tmp_path / "expected"
    exp.mkdir()
    expected_logs(exp, orig, recon, 27, prof=True)
    out, _ = run_cli(tmp_path, 416, 240, 3, 27, ("--prof",))
    assert len(compare_dirs(out, exp)) == 40
