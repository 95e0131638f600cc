"""Test helper: vectorised numpy backward search over the HOST arrays of an FmIndex.

Used only by the CPU tests to check the index layout (occ/runs/prefix) against the oracle without a
GPU. It reads the arrays through the C ABI accessor ``speq_index_array``; it is not part of the product path.
"""
from __future__ import annotations

import numpy as np

SYM = {ord("A"): 0, ord("C"): 1, ord("G"): 2, ord("T"): 3}
BLOCK = 96


def _popc32(x: np.ndarray) -> np.ndarray:
    return np.bitwise_count(x.astype(np.uint32)).astype(np.int64)


def entry_rank(entries: np.ndarray, idx: np.ndarray, r: np.ndarray) -> np.ndarray:
    """entries: (m, 4) u32 {count, bits0, bits1, bits2}; rank = count + popcount of the first r bits (0..96)."""
    e = entries[idx]
    out = e[:, 0].astype(np.int64)
    for w in range(3):
        lo = 32 * w
        full = r >= lo + 32
        part = (r > lo) & ~full
        bits = e[:, 1 + w].astype(np.uint64)
        sh = np.clip(r - lo, 0, 31).astype(np.uint64)
        mask = ((np.uint64(1) << sh) - np.uint64(1)).astype(np.uint64)
        out += np.where(full, _popc32(bits), 0) + np.where(part, _popc32(bits & mask), 0)
    return out


class NumpyFm:
    def __init__(self, index):
        self.occ = index.array("occ", np.uint32).reshape(-1, 4)       # (5*nb, 4): plane-major [symbol][block]
        self.nb = self.occ.shape[0] // 5
        self.runs = index.array("runs", np.uint32).reshape(-1, 4)
        self.run_label = index.array("run_label", np.uint16)
        self.C = index.array("C", np.uint32).astype(np.int64)
        self.n = int(index.info().n)
        self.q = int(index.info().prefix_q)
        self.prefix = index.array("prefix", np.uint32).reshape(-1, 2) if self.q else None
        lab = index.array("lab", np.uint32)
        self.lab = lab if lab.size else None
        occ2 = index.array("occ2", np.uint32)
        self.occ2 = occ2.reshape(-1, 4) if occ2.size else None
        occ3 = index.array("occ3", np.uint32)
        self.occ3 = occ3.reshape(-1, 4) if occ3.size else None

    def lf(self, sym: np.ndarray, i: np.ndarray) -> np.ndarray:
        """LF(sym, i) = C[sym] + rank; sym: 0..3 ACGT, 4 N (entry counts include C)."""
        b, r = i // BLOCK, i % BLOCK
        return entry_rank(self.occ, sym * self.nb + b, r)

    def lf2(self, a: np.ndarray, b: np.ndarray, i: np.ndarray) -> np.ndarray:
        """Two-symbol LF: interval of abP from that of P (plane 4a+b)."""
        blk, r = i // BLOCK, i % BLOCK
        return entry_rank(self.occ2, (a * 4 + b) * self.nb + blk, r)

    def lf3(self, a: np.ndarray, b: np.ndarray, c: np.ndarray, i: np.ndarray) -> np.ndarray:
        """Three-symbol LF: interval of abcP from that of P (plane 16a+4b+c)."""
        blk, r = i // BLOCK, i % BLOCK
        return entry_rank(self.occ3, (a * 16 + b * 4 + c) * self.nb + blk, r)

    def rank(self, sym: np.ndarray, i: np.ndarray) -> np.ndarray:
        return self.lf(sym, i) - self.C[np.asarray(sym) + 2]

    def run_of(self, i: np.ndarray) -> np.ndarray:
        return entry_rank(self.runs, i // BLOCK, i % BLOCK + 1)

    def classify(self, kmers: np.ndarray, use_prefix: bool = True, use_pairs: bool = True,
                 use_lab: bool = True, use_triples: bool = True) -> np.ndarray:
        """kmers: (m, k) symbols 0..4. Returns -1 / -2 / group per row (same contract as the kernel)."""
        m, k = kmers.shape
        lo = np.zeros(m, dtype=np.int64)
        hi = np.full(m, self.n, dtype=np.int64)
        start = k
        if use_prefix and self.q and k >= self.q:
            tail = kmers[:, k - self.q:]
            okq = (tail < 4).all(axis=1)
            code = np.zeros(m, dtype=np.int64)
            for j in range(self.q):
                code = code * 4 + (tail[:, j] & 3)
            lo = np.where(okq, self.prefix[code, 0].astype(np.int64), lo)
            hi = np.where(okq, self.prefix[code, 1].astype(np.int64), hi)
            steps = np.where(okq, k - self.q, k)
        else:
            steps = np.full(m, k)
        if self.occ3 is not None and use_triples:
            # remainder mod 3 first (one single or one pair step), then triples (same order as the kernel)
            ok = ~(kmers == 4).any(axis=1)
            steps = steps.copy()
            for rem in (1, 2):
                rows = np.nonzero((steps % 3 == rem) & (lo < hi) & ok)[0]
                if not rows.size:
                    continue
                if rem == 1:
                    c = kmers[rows, steps[rows] - 1].astype(np.int64)
                    lo[rows], hi[rows] = self.lf(c, lo[rows]), self.lf(c, hi[rows])
                else:
                    a = kmers[rows, steps[rows] - 2].astype(np.int64)
                    b = kmers[rows, steps[rows] - 1].astype(np.int64)
                    lo[rows], hi[rows] = self.lf2(a, b, lo[rows]), self.lf2(a, b, hi[rows])
                steps[rows] -= rem
            # windows that could not take multi-symbol steps (N) keep their single steps below
            single_steps = np.where(ok, 0, steps)
            steps = np.where(ok, steps, 0)
            while True:
                act = (steps > 0) & (lo < hi)
                if not act.any():
                    break
                rows = np.nonzero(act)[0]
                a = kmers[rows, steps[rows] - 3].astype(np.int64)
                b = kmers[rows, steps[rows] - 2].astype(np.int64)
                c = kmers[rows, steps[rows] - 1].astype(np.int64)
                lo[rows], hi[rows] = self.lf3(a, b, c, lo[rows]), self.lf3(a, b, c, hi[rows])
                steps[rows] -= 3
            steps = single_steps
        elif self.occ2 is not None and use_pairs:
            # odd remainder: one single step first, then pairs (same order as the kernel)
            pair_ok = ~(kmers == 4).any(axis=1)
            odd = (steps % 2 == 1) & (lo < hi) & pair_ok
            rows = np.nonzero(odd)[0]
            if rows.size:
                c = kmers[rows, steps[rows] - 1].astype(np.int64)
                lo[rows] = self.lf(c, lo[rows])
                hi[rows] = self.lf(c, hi[rows])
                steps = steps.copy()
                steps[rows] -= 1
            single_steps = np.where(pair_ok, 0, steps)
            steps = np.where(pair_ok, steps, 0)
            while True:
                act = (steps > 0) & (lo < hi)
                if not act.any():
                    break
                rows = np.nonzero(act)[0]
                a = kmers[rows, steps[rows] - 2].astype(np.int64)
                b = kmers[rows, steps[rows] - 1].astype(np.int64)
                lo[rows] = self.lf2(a, b, lo[rows])
                hi[rows] = self.lf2(a, b, hi[rows])
                steps[rows] -= 2
            steps = single_steps
        for s in range(start, 0, -1):
            act = (s <= steps) & (lo < hi)
            if not act.any():
                continue
            c = kmers[act, s - 1].astype(np.int64)
            lo[act] = self.lf(c, lo[act])
            hi[act] = self.lf(c, hi[act])
        out = np.full(m, -1, dtype=np.int64)
        hit = lo < hi
        if hit.any():
            rl = self.run_of(lo[hit])
            rh = self.run_of(hi[hit] - 1)
            by_runs = np.where(rl == rh, self.run_label[rl].astype(np.int64), -2)
            if self.lab is not None and use_lab:  # the kernel's one-load path must agree with the rank path
                x = self.lab[lo[hit]].astype(np.int64)
                dist, width = x >> 16, hi[hit] - lo[hit]
                by_lab = np.where(width <= dist, x & 0xFFFF, np.where(dist < 0xFFFF, -2, by_runs))
                assert np.array_equal(by_lab, by_runs)
            out[hit] = by_runs
        return out


def ascii_to_syms(b: bytes | np.ndarray) -> np.ndarray:
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else b
    lut = np.full(256, 4, dtype=np.int64)
    for ch, v in ((b"A", 0), (b"C", 1), (b"G", 2), (b"T", 3), (b"U", 3)):
        lut[ch[0]] = v
        lut[ch.lower()[0]] = v
    return lut[a]
