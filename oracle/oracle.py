"""ctypes wrapper of the CPU oracle (oracle/build/libkmer_oracle.so). TEST INFRASTRUCTURE ONLY.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg — never by speq_amd/.
See kmer_oracle.c for what it restates (and "parity unpinned" at the SeqAn3 boundary).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import time
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libkmer_oracle.so")
_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        U64P = C.POINTER(C.c_uint64)
        L.oracle_build.restype = P
        L.oracle_build.argtypes = [C.c_char_p, U64P, C.c_uint32, C.POINTER(C.c_int32), C.c_uint32, C.c_uint32]
        L.oracle_free.argtypes = [P]
        L.oracle_lookup_ascii.restype = C.c_int32
        L.oracle_lookup_ascii.argtypes = [P, C.c_char_p]
        L.oracle_scan.restype = C.c_int
        L.oracle_scan.argtypes = [P, C.c_char_p, C.c_char_p, U64P, C.c_uint64, C.c_int, C.c_uint32, C.c_int, U64P,
                                  C.POINTER(C.c_double), C.c_int]
        L.oracle_em_pass.restype = C.c_int
        L.oracle_em_pass.argtypes = [P, C.c_char_p, C.c_char_p, U64P, C.c_uint64, C.c_int, C.c_uint32, C.c_int,
                                     C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_int32), C.POINTER(C.c_double)]
        L.oracle_ref_unique.restype = C.c_int
        L.oracle_ref_unique.argtypes = [P, U64P, U64P]
        L.sl_build.restype = P
        L.sl_build.argtypes = [C.c_char_p, U64P, C.c_uint32, C.POINTER(C.c_int32), C.c_uint32]
        L.sl_build_sa.restype = P
        L.sl_build_sa.argtypes = [C.c_char_p, U64P, C.c_uint32, C.POINTER(C.c_int32), C.c_uint32,
                                  C.POINTER(C.c_uint32)]
        L.sl_sample.restype = C.c_uint32
        L.sl_sample.argtypes = [P, C.c_uint32]
        L.sl_free.argtypes = [P]
        L.sl_count.restype = C.c_int64
        L.sl_count.argtypes = [P, C.c_char_p, C.c_uint32]
        L.sl_which.restype = C.c_int32
        L.sl_which.argtypes = [P, C.c_char_p, C.c_uint32]
        L.sl_scan.restype = C.c_int
        L.sl_scan.argtypes = [P, C.c_char_p, C.c_char_p, U64P, C.c_uint64, C.c_int, C.c_uint32, C.c_uint32, C.c_int,
                              U64P, C.POINTER(C.c_double), C.c_int]
        L.sl_text_len.restype = C.c_uint32
        L.sl_text_len.argtypes = [P]
        L.fmcpu_scan.restype = C.c_int
        L.fmcpu_scan.argtypes = [C.POINTER(FmCpuView), C.c_char_p, C.c_char_p, U64P, C.c_uint64, C.c_int, C.c_uint32,
                                 C.c_uint32, U64P, C.c_int]
        _lib = L
    return _lib


def _u64p(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


class Oracle:
    """k-mer -> group-label hash map over [fwd_r, rc_r] of every record."""

    def __init__(self, records: Sequence[bytes], groups: Sequence[int], n_groups: int, k: int):
        bs = [bytes(r) for r in records]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        g = np.asarray(groups, dtype=np.int32)
        self.k, self.G = k, n_groups
        self._h = lib().oracle_build(b"".join(bs), _u64p(off), len(bs), g.ctypes.data_as(C.POINTER(C.c_int32)),
                                     n_groups, k)
        if not self._h:
            raise ValueError("oracle_build failed")

    def lookup(self, kmer: bytes) -> int:
        assert len(kmer) == self.k
        return int(lib().oracle_lookup_ascii(self._h, kmer))

    def scan(self, seq, qual, offsets, phred_cutoff: int = 30, paired: bool = False, local: bool = False,
             threads: int = 0):
        """Returns (T, ambiguous, U[G] u64, W[G] f64 or None)."""
        seq_b = seq.tobytes() if isinstance(seq, np.ndarray) else bytes(seq)
        qual_b = qual.tobytes() if isinstance(qual, np.ndarray) else bytes(qual)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        counts = np.zeros(self.G + 2, dtype=np.uint64)
        w = np.zeros(self.G, dtype=np.float64) if local else None
        rc = lib().oracle_scan(self._h, seq_b, qual_b, _u64p(off), len(off) - 1, int(paired), phred_cutoff,
                               1 if local else 0, _u64p(counts),
                               w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None, threads)
        if rc != 0:
            raise ValueError("oracle_scan: bad arguments")
        return int(counts[0]), int(counts[1]), counts[2:].copy(), w

    def em_pass(self, seq, qual, offsets, percent, group_counts, phred_cutoff: int = 30, paired: bool = False,
                local: bool = False, percent_perfect: float = 1.0):
        """One literal EM estimator pass of the reference; returns next_tkpg[G]."""
        seq_b = seq.tobytes() if isinstance(seq, np.ndarray) else bytes(seq)
        qual_b = qual.tobytes() if isinstance(qual, np.ndarray) else bytes(qual)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        p = np.ascontiguousarray(percent, dtype=np.float64)
        gc = np.ascontiguousarray(group_counts, dtype=np.int32)
        nxt = np.zeros(self.G, dtype=np.float64)
        dp = C.POINTER(C.c_double)
        rc = lib().oracle_em_pass(self._h, seq_b, qual_b, _u64p(off), len(off) - 1, int(paired), phred_cutoff,
                                  1 if local else 0, percent_perfect, p.ctypes.data_as(dp),
                                  gc.ctypes.data_as(C.POINTER(C.c_int32)), nxt.ctypes.data_as(dp))
        if rc != 0:
            raise ValueError("oracle_em_pass: bad arguments")
        return nxt

    def ref_unique(self):
        u = np.zeros(self.G, dtype=np.uint64)
        t = np.zeros(self.G, dtype=np.uint64)
        lib().oracle_ref_unique(self._h, _u64p(u), _u64p(t))
        return u, t

    def __del__(self):
        try:
            if self._h:
                lib().oracle_free(self._h)
                self._h = None
        except Exception:
            pass


class SeqanLike:
    """CPU stand-in for the reference's algorithm (seqan_like.c): backward search on a wavelet structure, locate of
    every hit through SA samples (every 16 rows), sorted hit list, first-hit group rule. k is chosen per scan, as
    with the reference's index."""

    def __init__(self, records: Sequence[bytes], groups: Sequence[int], n_groups: int, sa=None):
        """sa: optional suffix array of the same text (t_0 $ t_1 $ ... #, codes # $ A C G T N = 0..6), e.g. the
        product index's (FmIndex.array("sa")): a suffix array is unique, so it only skips this file's own O(n log n)
        sort (bench.py's config-5 baseline; the scan, which is what is timed, is this file's code alone)."""
        bs = [bytes(r) for r in records]
        off = np.zeros(len(bs) + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(b) for b in bs])
        g = np.asarray(groups, dtype=np.int32)
        self.G = n_groups
        if sa is None:
            self._h = lib().sl_build(b"".join(bs), _u64p(off), len(bs), g.ctypes.data_as(C.POINTER(C.c_int32)),
                                     n_groups)
        else:
            sa = np.ascontiguousarray(sa, dtype=np.uint32)
            if len(sa) != int(off[-1]) * 2 + 2 * len(bs) + 1:
                raise ValueError("SeqanLike: suffix array length does not match the text")
            self._h = lib().sl_build_sa(b"".join(bs), _u64p(off), len(bs), g.ctypes.data_as(C.POINTER(C.c_int32)),
                                        n_groups, sa.ctypes.data_as(C.POINTER(C.c_uint32)))
        if not self._h:
            raise ValueError("sl_build failed")

    @property
    def n(self) -> int:
        return int(lib().sl_text_len(self._h))

    def count(self, kmer: bytes) -> int:
        return int(lib().sl_count(self._h, kmer, len(kmer)))

    def sample(self, j: int) -> int:
        """SA[16 j] of this structure (0xFFFFFFFF past the end)."""
        return int(lib().sl_sample(self._h, j))

    def which(self, kmer: bytes) -> int:
        return int(lib().sl_which(self._h, kmer, len(kmer)))

    def scan(self, seq, qual, offsets, k: int, phred_cutoff: int = 30, paired: bool = False, local: bool = False,
             threads: int = 0):
        """Returns (T, ambiguous, U[G] u64, W[G] f64 or None)."""
        seq_b = seq.tobytes() if isinstance(seq, np.ndarray) else bytes(seq)
        qual_b = qual.tobytes() if isinstance(qual, np.ndarray) else bytes(qual)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        counts = np.zeros(self.G + 2, dtype=np.uint64)
        w = np.zeros(self.G, dtype=np.float64) if local else None
        rc = lib().sl_scan(self._h, seq_b, qual_b, _u64p(off), len(off) - 1, int(paired), k, phred_cutoff,
                           1 if local else 0, _u64p(counts),
                           w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None, threads)
        if rc != 0:
            raise ValueError("sl_scan: bad arguments")
        return int(counts[0]), int(counts[1]), counts[2:].copy(), w

    def __del__(self):
        try:
            if self._h:
                lib().sl_free(self._h)
                self._h = None
        except Exception:
            pass


class FmCpuView(C.Structure):
    _fields_ = [("occ", C.c_void_p), ("occ2", C.c_void_p), ("occ3", C.c_void_p), ("runs", C.c_void_p),
                ("run_label", C.c_void_p), ("prefix", C.c_void_p * 3), ("q", C.c_uint32), ("n", C.c_uint32),
                ("nb", C.c_uint32), ("G", C.c_uint32)]


class FmCpu:
    """The build's own label-run algorithm on host cores (fm_cpu.c) over the arrays of a built speq_amd index."""

    def __init__(self, index):
        info = index.info()
        self._keep = {}

        def arr(name, dt):
            a = index.array(name, dt)
            self._keep[name] = a
            return a.ctypes.data if a.size else None

        v = FmCpuView()
        v.occ, v.occ2, v.occ3 = arr("occ", np.uint32), arr("occ2", np.uint32), arr("occ3", np.uint32)
        v.runs, v.run_label = arr("runs", np.uint32), arr("run_label", np.uint16)
        for i, name in enumerate(("prefix", "prefix_q1", "prefix_q2")):
            v.prefix[i] = arr(name, np.uint32)
        v.q, v.n, v.G = info.prefix_q, info.n, info.n_groups
        v.nb = info.n // 96 + 1
        self.view, self.G = v, info.n_groups

    def scan(self, seq, qual, offsets, k: int, phred_cutoff: int = 30, paired: bool = False, threads: int = 0):
        seq_b = seq.tobytes() if isinstance(seq, np.ndarray) else bytes(seq)
        qual_b = qual.tobytes() if isinstance(qual, np.ndarray) else bytes(qual)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        counts = np.zeros(self.G + 2, dtype=np.uint64)
        rc = lib().fmcpu_scan(C.byref(self.view), seq_b, qual_b, _u64p(off), len(off) - 1, int(paired), k,
                              phred_cutoff, _u64p(counts), threads)
        if rc != 0:
            raise ValueError("fmcpu_scan: bad arguments (k must be <= 32)")
        return int(counts[0]), int(counts[1]), counts[2:].copy()


def time_scan(oracle: Oracle, seq, qual, offsets, threads: int = 0, min_seconds: float = 0.0):
    """Times oracle.scan (the CPU baseline leg of bench.py). Returns (seconds, result)."""
    t0 = time.perf_counter()
    res = oracle.scan(seq, qual, offsets, threads=threads)
    return time.perf_counter() - t0, res
