"""Device-side entry points (HIP kernels via libvame.so) on torch.cuda tensors.

Mirrors the reference's operator interface for this path:
  * `Engine.affine_me(ref, cur, lam, align, ncp, extra, prev)` == one launch of
    affine_gradient_mult_sizes(_HA) built with -DnCP=ncp (affine.cl:11/:960,
    args set at main.cpp:827-840), returning the gBestCost / gBestCpmvs arrays;
  * `Engine.affine_me_poc(cur, refs, lam, ...)` == the whole refIdx loop of one
    POC (main.cpp:746-966), fused into one pass;
  * `Engine.affine_me_batch([(cur, refs, lam, out), ...])` == several POCs'
    affine_me_poc calls in shared launches.
Frames are (H, W) int16/uint16 tensors of 10-bit samples on the engine's device.
"""
from __future__ import annotations

import ctypes

import torch

from ._lib import PocJob, PocResult, check, lib

CPMV_FIELDS = ("nCPs", "LTx", "LTy", "RTx", "RTy", "LBx", "LBy")
MODES = ("FULL_2CP", "FULL_3CP", "HALF_2CP", "HALF_3CP")
# mode_mask bits (include/vame.h): 2-CP, 3-CP, and the alignment selection
MODE_2CP, MODE_3CP, MODE_FULL, MODE_HALF = 1, 2, 4, 8


def pred_mask(modes: int) -> int:
    """vame_pred_mask: the PREDs (bit m of MODES) a mode mask codes."""
    ncp = 3 if modes & MODE_3CP else 1
    sel = (modes >> 2) & 3
    return (ncp if sel in (0, 1, 3) else 0) | ((ncp << 2) if sel in (0, 2, 3) else 0)


def _ptr(t: torch.Tensor | None):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


class Engine:
    def __init__(self, width: int, height: int, device: int | torch.device = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("vame.Engine needs a HIP device (no CPU fallback)")
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index)
        self.W, self.H = width, height
        self.n_ctus = lib().vame_num_ctus(width, height)
        if not self.n_ctus:
            raise ValueError(f"unsupported resolution {width}x{height}")
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            check(lib().vame_create(ctypes.byref(h), self.device.index, width, height))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().vame_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_prof(self, enable: bool) -> None:
        """PROF on/off for later launches (the reference hard-disables it,
        affine.cl:168); vame_set_prof."""
        check(lib().vame_set_prof(self._h, int(enable)))

    def set_max_pairs(self, n: int) -> None:
        """(POC, refIdx) pairs per launch, 1..32 (default 32): sizes the
        context's 3-CP seed-reuse scratch (vame_set_max_pairs)."""
        check(lib().vame_set_max_pairs(self._h, int(n)))

    @property
    def max_pairs(self) -> int:
        return lib().vame_get_max_pairs(self._h)

    def set_timing(self, enable, keep: bool = False) -> None:
        """True / 1: time every kernel class; 2: the quadrant kernel only; 0: off.
        keep: leave the launches recorded so far (VAME_TIMING_KEEP)."""
        check(lib().vame_set_timing(self._h, int(enable) | (16 if keep else 0)))

    def get_timing(self, kernel_class: int, reset: bool = True):
        """(total_ms, launches) of kernel class 0 (quadrant items, affine_me_quad) /
        3 (128x128 CUs, affine_me_ctu2) / 4, 5 (128x64 / 64x128 CUs,
        affine_me_half2w / affine_me_half2h); under PROF 1 (128x128 CUs,
        affine_me_ctu_prof) / 2 (128x64 and 64x128 CUs, affine_me_half_prof)."""
        t, n = ctypes.c_double(), ctypes.c_int()
        check(lib().vame_get_timing(self._h, kernel_class, ctypes.byref(t), ctypes.byref(n), int(reset)))
        return t.value, n.value

    def n_cus(self, align: int) -> int:
        return self.n_ctus * (284 if align else 201)

    def _frame(self, f: torch.Tensor) -> torch.Tensor:
        if f.shape != (self.H, self.W) or f.device != self.device or f.dtype not in (torch.int16, torch.uint16):
            raise ValueError(f"frame must be ({self.H},{self.W}) int16/uint16 on {self.device}")
        return f.contiguous()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _check_out(self, out, align: int):
        """Caller-supplied result buffers must hold exactly the launch's rows:
        int64 cost[n], int32 cpmv[n, 7], contiguous, on the engine's device."""
        cost, cpmv = out
        n = self.n_cus(align)
        ok = (cost.dtype == torch.int64 and cost.numel() == n and cost.is_contiguous()
              and cpmv.dtype == torch.int32 and tuple(cpmv.shape) == (n, 7) and cpmv.is_contiguous()
              and cost.device == self.device and cpmv.device == self.device)
        if not ok:
            raise ValueError(f"result buffers must be int64[{n}] and int32[{n}, 7], contiguous, "
                             f"on {self.device} (align={align})")
        return cost, cpmv

    def alloc_result(self, align: int):
        n = self.n_cus(align)
        return (torch.empty(n, dtype=torch.int64, device=self.device),
                torch.empty((n, 7), dtype=torch.int32, device=self.device))

    def affine_me(self, ref, cur, lam: float, align: int, ncp: int, extra: int = 0,
                  prev: torch.Tensor | None = None, out=None):
        ref, cur = self._frame(ref), self._frame(cur)
        if align not in (0, 1) or ncp not in (2, 3):
            raise ValueError("align must be 0/1 and ncp 2/3")
        cost, cpmv = self._check_out(out, align) if out is not None else self.alloc_result(align)
        if ncp == 3 and (prev is None or tuple(prev.shape) != (self.n_cus(align), 7)
                         or prev.dtype != torch.int32 or prev.device != self.device):
            raise ValueError("3-CP needs prev = the same-alignment 2-CP cpmvs, int32 [n, 7] on the device")
        check(lib().vame_affine_me(self._h, _ptr(ref), _ptr(cur), float(lam), align, ncp, extra,
                                   _ptr(prev.contiguous()) if prev is not None else None,
                                   _ptr(cost), _ptr(cpmv), self._stream()))
        return cost, cpmv

    def alloc_poc(self, nrefs: int, modes: int = 3):
        res = {}
        preds = pred_mask(modes)
        for r in range(nrefs):
            for m, name in enumerate(MODES):
                if (preds >> m) & 1:
                    res[(r, name)] = self.alloc_result(m >> 1)
        return res

    def _check_poc_out(self, out, nrefs: int, modes: int):
        preds = pred_mask(modes)
        need = {(r, name) for r in range(nrefs) for m, name in enumerate(MODES) if (preds >> m) & 1}
        missing = need - set(out)
        if missing:
            raise ValueError(f"result buffers missing for {sorted(missing)}")
        for (r, name), bufs in out.items():
            if r >= nrefs or name not in MODES:
                raise ValueError(f"unexpected result key {(r, name)}")
            self._check_out(bufs, MODES.index(name) >> 1)

    def affine_me_batch(self, jobs, modes: int = 3, extra: int = 0):
        """jobs: [(cur, refs, lam, out)] with out from alloc_poc; one
        vame_affine_me_batch call (max_pairs (POC, refIdx) pairs per launch,
        default 32)."""
        keep = []
        arr = (PocJob * len(jobs))()
        for j, (cur, refs, lam, out) in enumerate(jobs):
            cur = self._frame(cur)
            refs = [self._frame(r) for r in refs]
            self._check_poc_out(out, len(refs), modes)
            pr = PocResult()
            for (r, name), (cost, cpmv) in out.items():
                m = MODES.index(name)
                pr.cost[r][m] = cost.data_ptr()
                pr.cpmvs[r][m] = cpmv.data_ptr()
            ref_ptrs = (ctypes.c_void_p * len(refs))(*[r.data_ptr() for r in refs])
            keep += [cur, refs, pr, ref_ptrs]
            arr[j].cur = cur.data_ptr()
            arr[j].refs = ctypes.cast(ref_ptrs, ctypes.c_void_p)
            arr[j].nrefs = len(refs)
            arr[j].lam = float(lam)
            arr[j].out = ctypes.cast(ctypes.pointer(pr), ctypes.c_void_p)
        check(lib().vame_affine_me_batch(self._h, arr, len(jobs), modes, extra, self._stream()))
        return [job[3] for job in jobs]

    def pack_records(self, results: list[dict], modes: int, words: int | None = None,
                     bad: torch.Tensor | None = None) -> torch.Tensor:
        """vame_pack_records: the POCs' results (alloc_poc dicts, POC order) in
        the compact wire form of shard.pack, one kernel, zero-padded to
        `words`; `bad` (int32 device scalar) is OR-ed with 1 when a record does
        not fit the form (shard.check_flag reads it)."""
        from .shard import slab_words
        need = slab_words([(max(r for r, _ in res) + 1, modes, (self.n_cus(0), self.n_cus(1)))
                           for res in results])
        words = need if words is None else words
        if words < need:
            raise ValueError("slab larger than the agreed size")
        slab = torch.empty(words, dtype=torch.int32, device=self.device)
        if bad is None:
            bad = torch.zeros((), dtype=torch.int32, device=self.device)
        arr = (PocJob * max(len(results), 1))()
        keep = []
        for j, res in enumerate(results):
            nrefs = max(r for r, _ in res) + 1
            self._check_poc_out(res, nrefs, modes)
            pr = PocResult()
            for (r, name), (cost, cpmv) in res.items():
                m = MODES.index(name)
                pr.cost[r][m] = cost.data_ptr()
                pr.cpmvs[r][m] = cpmv.data_ptr()
            keep.append(pr)
            arr[j].nrefs = nrefs
            arr[j].out = ctypes.cast(ctypes.pointer(pr), ctypes.c_void_p)
        check(lib().vame_pack_records(self._h, arr, len(results), modes, slab.data_ptr(), words,
                                      bad.data_ptr(), self._stream()))
        return slab

    def affine_me_poc(self, cur, refs, lam: float, modes: int = 3, extra: int = 0, out=None):
        """modes: 1 = 2-CP only, 3 = 2-CP then 3-CP, plus MODE_FULL / MODE_HALF to
        code one alignment only.  Returns {(refIdx, MODE): (cost, cpmv)}."""
        cur = self._frame(cur)
        refs = [self._frame(r) for r in refs]
        out = out if out is not None else self.alloc_poc(len(refs), modes)
        self._check_poc_out(out, len(refs), modes)
        pr = PocResult()
        for (r, name), (cost, cpmv) in out.items():
            m = MODES.index(name)
            pr.cost[r][m] = cost.data_ptr()
            pr.cpmvs[r][m] = cpmv.data_ptr()
        ref_ptrs = (ctypes.c_void_p * len(refs))(*[r.data_ptr() for r in refs])
        check(lib().vame_affine_me_poc(self._h, _ptr(cur), ref_ptrs, len(refs), float(lam), modes,
                                       extra, ctypes.byref(pr), self._stream()))
        return out
