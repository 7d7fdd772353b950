"""The native sequence generator (csrc/vame_synth.c) produces the same bytes as
its numpy specification (vame/synth.py), so every config's frames are defined
by the numpy code whichever implementation made them."""
import numpy as np
import pytest

from vame import synth

pytestmark = pytest.mark.skipif(synth.native() is None, reason="libvame_synth.so not built")


@pytest.mark.parametrize("W,H,poc,seed", [(416, 240, 0, 0x5EED), (416, 240, 7, 0x5EED),
                                          (832, 480, 30, 0x5EED + 7919), (200, 136, 239, 12345)])
def test_native_frame_equals_numpy(W, H, poc, seed):
    a = synth.synth_frame(W, H, poc, seed)
    b = synth.synth_frame_np(W, H, poc, seed)
    assert a.dtype == b.dtype == np.uint16 and (a == b).all()
    assert 0 < (a == 600).mean() < 0.5  # the flat patch is there
    assert a.std() > 50  # and texture


@pytest.mark.parametrize("qp", [17, 22, 32, 37])
def test_native_recon_equals_numpy(qp):
    f = synth.synth_frame(416, 240, 3)
    a = synth.recon_frame(f, 3, qp)
    b = synth.recon_np(f, 3, qp)
    assert (a == b).all()
    d = a.astype(int) - f
    amp = synth.recon_noise_amp(qp)
    assert np.abs(d).max() <= amp and (amp == 0 or (d != 0).mean() > 0.5)


def test_sequence_and_shard_frames_agree():
    o, r = synth.synth_sequence(416, 240, 6, 27)
    assert (o[2] == synth.synth_frame(416, 240, 3)).all()
    oo, rr = synth.synth_pocs(416, 240, [4, 5], [0, 3, 4], 27)
    assert (oo[4] == o[3]).all() and (oo[5] == o[4]).all()
    for p in (0, 3, 4):
        assert (rr[p] == r[p]).all()


def test_native_csv_equals_numpy_writer(tmp_path):
    fr = synth.synth_sequence(64, 24, 2)[0]
    a, b = tmp_path / "a.csv", tmp_path / "b.csv"
    synth.write_csv(str(a), fr)
    with open(b, "w") as f:
        for k in range(fr.shape[0]):
            np.savetxt(f, fr[k], fmt="%d", delimiter=",")
    assert a.read_bytes() == b.read_bytes()
