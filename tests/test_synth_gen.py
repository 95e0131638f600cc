"""tools/synth_gen.c (the multithreaded read generator bench.py uses) against synth.py's numpy definition."""
import numpy as np
import pytest

from speq_amd import synth


@pytest.mark.parametrize("kw", [
    dict(),
    dict(n_rate=0.01, lowq_rate=0.02, short_frac=0.1),
    dict(paired=True),
    dict(paired=True, n_rate=0.005, short_frac=0.05, fragment=250),
])
def test_native_reads_match_numpy(kw, monkeypatch):
    ref = synth.make_reference(7, 2, 3000)
    if synth._synth_lib() is None:
        pytest.skip("tools/build/libsynth_gen.so not built")
    got = synth.make_reads(ref, 1500, start_index=123, **kw)
    monkeypatch.setenv("SPEQ_SYNTH_NUMPY", "1")
    monkeypatch.setattr(synth, "_SYNTH_LIB", None)
    exp = synth.make_reads(ref, 1500, start_index=123, chunk=700, **kw)
    assert np.array_equal(got.seq, exp.seq)
    assert np.array_equal(got.qual, exp.qual)
    assert np.array_equal(got.offsets, exp.offsets)
    assert np.array_equal(got.variant, exp.variant)


def test_native_reads_reference_with_n():
    ref = synth.make_reference(3, 1, 2000, ref_n_rate=0.01)
    if synth._synth_lib() is None:
        pytest.skip("tools/build/libsynth_gen.so not built")
    got = synth.make_reads(ref, 800, err_rate=0.05)
    synth._SYNTH_LIB = None
    import os
    os.environ["SPEQ_SYNTH_NUMPY"] = "1"
    try:
        exp = synth.make_reads(ref, 800, err_rate=0.05)
    finally:
        del os.environ["SPEQ_SYNTH_NUMPY"]
        synth._SYNTH_LIB = None
    assert np.array_equal(got.seq, exp.seq) and np.array_equal(got.offsets, exp.offsets)
