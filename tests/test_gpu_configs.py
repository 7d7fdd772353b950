"""BASELINE.json configs on the HIP path (libvame.so through the C ABI), with the
reference's own sequence semantics: the 4-slot reference ring with long-term
references (main.cpp:591-707, `hostlogic.ref_list`) and the per-POC QP offset
of the GOP-8 model (main_aux_functions.h:1482-1497, `hostlogic.lambda_for_poc`:
POC = 0 mod 8 codes at QP+1).  Every sampled (POC, refIdx) pair is compared
bit for bit -- every cost and every CPMV component of every candidate CU, all
four PRED modes -- against the pinned CPU oracle; the remaining pairs of each
sequence are checked against the per-POC entry point on the device.

  configs[1] C2  1920x1080 QP32, 2 frames, 2-CP only (mode_mask 1): all 3 pairs
  configs[2] C3  1920x1080 QP32, 30 frames, 2+3 CP: 114 pairs in one batched
                 call, 12 pairs spanning POC 1-30 vs the oracle
  configs[3] C4  3840x2160 at QP 22/27/32/37 (the QP changes the recon noise
                 and lambda): POCs 8 and 9 (long-term ref POC 0 / POC 8, the
                 QP+1 lambda of POC 8) per QP, and the whole 30-frame ring at
                 QP32
  configs[4] C5  3840x2160 QP32, 240 frames sharded by POC over 8 GPUs: the
                 last rank's block (POC 211-240, `shard.poc_shard(240, 8, 7)`)
                 in one batched call -- the ring's long-term references at
                 high POCs (POC 239: 238 232 224 216) and the QP+1 lambda of
                 POC 240 -- three pairs vs the oracle, POCs vs per-POC calls
"""
import numpy as np
import pytest
import torch

import oracle_py as O

pytestmark = pytest.mark.gpu

MODES = {"FULL_2CP": (0, 2), "FULL_3CP": (0, 3), "HALF_2CP": (1, 2), "HALF_3CP": (1, 3)}
FIELDS = ("LTx", "LTy", "RTx", "RTy", "LBx", "LBy")


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda()


def run_sequence(eng, orig, recon, qp, pocs, modes):
    """vame_affine_me_batch over `pocs` with the reference's refs and lambdas.
    orig / recon: {poc: frame} (orig POC p, reconstructed POC p)."""
    from vame.hostlogic import lambda_for_poc, ref_list
    d_recon = {p: dev(f) for p, f in recon.items()}
    jobs = []
    for poc in pocs:
        refs = ref_list(poc)
        jobs.append((dev(orig[poc]), [d_recon[r] for r in refs], lambda_for_poc(qp, poc),
                     eng.alloc_poc(len(refs), modes)))
    eng.affine_me_batch(jobs, modes, 0)
    torch.cuda.synchronize()
    return {poc: job for poc, job in zip(pocs, jobs)}


def check_pair_vs_oracle(job, refidx, ref_frame, cur_frame, modes, tag):
    _, _, lam, out = job
    want = O.affine_me_pair(ref_frame, cur_frame, lam, modes=(2, 3) if modes & 2 else (2,))
    for name, key in MODES.items():
        if key not in want:
            assert (refidx, name) not in out
            continue
        cost, cp = out[(refidx, name)]
        hc, hp = cost.cpu().numpy(), cp.cpu().numpy()
        oc, op = want[key]
        np.testing.assert_array_equal(hc, oc, err_msg=f"{tag} {name} cost")
        np.testing.assert_array_equal(hp[:, 1:], np.stack([op[f] for f in FIELDS], 1),
                                      err_msg=f"{tag} {name} cpmv")
        assert (hp[:, 0] == key[1]).all(), f"{tag} {name} nCPs"


def check_batch_vs_per_poc(eng, seq, d_orig, d_recon, modes):
    """Every pair of the batched call == one vame_affine_me_poc per POC (on the device)."""
    for poc, (cur, refs, lam, out) in seq.items():
        single = eng.affine_me_poc(cur, refs, lam, modes=modes)
        for key, (c, p) in out.items():
            sc, sp = single[key]
            assert torch.equal(c, sc) and torch.equal(p, sp), f"POC {poc} {key}"


@pytest.fixture(scope="module")
def engines():
    from vame.engine import Engine
    cache = {}

    def get(W, H):
        if (W, H) not in cache:
            cache[(W, H)] = Engine(W, H, 0)
        return cache[(W, H)]
    yield get
    for e in cache.values():
        e.close()


def test_c2_2cp_only_1080p(engines):
    """configs[1], the benchmarked workload: POC 1-2 (3 pairs), mode_mask 1."""
    from vame import synth
    o, r = synth.synth_sequence(1920, 1080, 2, 32)
    eng = engines(1920, 1080)
    seq = run_sequence(eng, {1: o[0], 2: o[1]}, {0: r[0], 1: r[1]}, 32, [1, 2], 1)
    from vame.hostlogic import ref_list
    for poc, job in seq.items():
        assert set(job[3]) == {(k, m) for k in range(len(job[1])) for m in ("FULL_2CP", "HALF_2CP")}
        for refidx, rp in enumerate(ref_list(poc)):
            check_pair_vs_oracle(job, refidx, r[rp], o[poc - 1], 1, f"POC{poc} ref{refidx}")


@pytest.fixture(scope="module")
def c3_run(engines):
    from vame import synth
    o, r = synth.synth_sequence(1920, 1080, 30, 32)
    eng = engines(1920, 1080)
    orig = {p: o[p - 1] for p in range(1, 31)}
    recon = {p: r[p] for p in range(30)}
    seq = run_sequence(eng, orig, recon, 32, list(range(1, 31)), 3)
    return eng, orig, recon, seq


# (POC, refIdx): short ring (POC 1-3), long-term POC 0 (POC 5, 8), the QP+1
# lambda of POC 8 / 16 / 24, long-term POC 8 (POC 12, 26) and 16 (POC 19)
C3_PAIRS = [(1, 0), (3, 2), (5, 3), (8, 0), (8, 3), (12, 2), (16, 1), (19, 1), (24, 0),
            (26, 3), (30, 0), (30, 2)]


@pytest.mark.parametrize("poc,refidx", C3_PAIRS, ids=[f"poc{p}_ref{k}" for p, k in C3_PAIRS])
def test_c3_1080p_30_frames_vs_oracle(c3_run, poc, refidx):
    from vame.hostlogic import ref_list
    eng, orig, recon, seq = c3_run
    assert sum(len(j[1]) for j in seq.values()) == 114
    rp = ref_list(poc)[refidx]
    check_pair_vs_oracle(seq[poc], refidx, recon[rp], orig[poc], 3, f"C3 POC{poc} ref{refidx}(POC{rp})")


def test_c3_batch_equals_per_poc(c3_run):
    eng, orig, recon, seq = c3_run
    check_batch_vs_per_poc(eng, seq, None, None, 3)


@pytest.mark.parametrize("qp,pairs", [(22, [(8, 3), (9, 1)]), (27, [(9, 0), (8, 1)]),
                                      (32, [(8, 0), (9, 3)]), (37, [(9, 2), (8, 3)])])
def test_c4_2160p_qp_sweep_vs_oracle(engines, qp, pairs):
    """configs[3] at every QP of the sweep: POC 8 (QP+1 lambda, refs 7 6 5 + long-term 0)
    and POC 9 (refs 8 7 6 0) in one batch, two pairs per QP vs the oracle."""
    from vame import synth
    from vame.hostlogic import ref_list
    pocs = [8, 9]
    refs = sorted({p for poc in pocs for p in ref_list(poc)})
    orig, recon = synth.synth_pocs(3840, 2160, pocs, refs, qp)
    eng = engines(3840, 2160)
    seq = run_sequence(eng, orig, recon, qp, pocs, 3)
    for poc, refidx in pairs:
        rp = ref_list(poc)[refidx]
        check_pair_vs_oracle(seq[poc], refidx, recon[rp], orig[poc], 3,
                             f"C4 QP{qp} POC{poc} ref{refidx}(POC{rp})")


def test_c4_2160p_30_frame_ring(engines):
    """configs[3] at QP32 with the whole 30-frame ring in one batched call
    (114 pairs at 3840x2160): the batch equals the per-POC calls, and the last
    POC's long-term pairs equal the oracle."""
    from vame import synth
    from vame.hostlogic import ref_list
    o, r = synth.synth_sequence(3840, 2160, 30, 32)
    eng = engines(3840, 2160)
    orig = {p: o[p - 1] for p in range(1, 31)}
    recon = {p: r[p] for p in range(30)}
    seq = run_sequence(eng, orig, recon, 32, list(range(1, 31)), 3)
    check_batch_vs_per_poc(eng, {p: seq[p] for p in (1, 8, 16, 29, 30)}, None, None, 3)
    for poc, refidx in ((30, 3), (24, 1)):
        rp = ref_list(poc)[refidx]
        check_pair_vs_oracle(seq[poc], refidx, recon[rp], orig[poc], 3, f"C4 ring POC{poc} ref{refidx}(POC{rp})")


def test_c5_2160p_last_shard_vs_oracle(engines):
    """configs[4]: the block the 8th GPU codes of the 240-frame 4K sequence,
    exactly as bench.py --config c5 --gpus 8 hands it to rank 7."""
    from vame import synth
    from vame.hostlogic import ref_list
    from vame.shard import poc_shard
    pocs = poc_shard(240, 8, 7)
    assert pocs[0] > 200 and pocs[-1] == 240
    refs = sorted({p for poc in pocs for p in ref_list(poc)})
    orig, recon = synth.synth_pocs(3840, 2160, pocs, refs, 32)
    eng = engines(3840, 2160)
    seq = run_sequence(eng, orig, recon, 32, pocs, 3)
    assert ref_list(239) == [238, 232, 224, 216]
    check_batch_vs_per_poc(eng, {p: seq[p] for p in (pocs[0], 232, 239, 240)}, None, None, 3)
    for poc, refidx in ((240, 0), (239, 3), (pocs[0], 2)):
        rp = ref_list(poc)[refidx]
        check_pair_vs_oracle(seq[poc], refidx, recon[rp], orig[poc], 3, f"C5 POC{poc} ref{refidx}(POC{rp})")
