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


def test_quality_profiles(monkeypatch):
    """apply_quality_profile: the native 'variable' generator writes the numpy definition's bytes; 'binned' uses the
    four NovaSeq bins only; both leave the bases alone."""
    ref = synth.make_reference(3, 1, 5_000)
    reads = synth.make_reads(ref, 3_000, short_frac=0.1)
    var = synth.apply_quality_profile(reads, "variable")
    monkeypatch.setenv("SPEQ_SYNTH_NUMPY", "1")
    monkeypatch.setattr(synth, "_SYNTH_LIB", None)
    var_np = synth.apply_quality_profile(reads, "variable")
    assert np.array_equal(var.qual, var_np.qual) and np.array_equal(var.seq, reads.seq)
    q = var.qual.astype(int) - 33
    assert q.min() >= 2 and q.max() <= 41 and 0.01 < (q <= 30).mean() < 0.06 and len(np.unique(q)) > 10
    b = synth.apply_quality_profile(reads, "binned").qual.astype(int) - 33
    assert set(np.unique(b).tolist()) <= {2, 12, 23, 37} and (b == 37).mean() > 0.8
    assert synth.apply_quality_profile(reads, "q40") is reads
