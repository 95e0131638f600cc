"""Python host mirror of the SPeQ scan path (thin layer over the C ABI in include/speq_scan.h).

Names follow the reference (``/root/reference``):

* :func:`file_to_map`       — ``speq::file_to_map``                      src/file_to_map.cpp:20-119
* :class:`FmIndex`          — ``seqan3::fm_index`` built by ``speq::fm::generate_fm_index``
                              src/fm_indexer.cpp:8-52 (texts [fwd_r, rc_r], :25-33)
* :meth:`DeviceIndex.scan`  — ``search`` + ``do_a_count`` over all reads  src/fm_scanner.cpp:137-236
* :meth:`DeviceIndex.count_unique_kmers_per_group`
                            — ``_async_count_unique_kmers_per_group``     src/fm_scanner.cpp:1476-1576
* :func:`unique_to_percent` — ``speq::scan::unique_to_percent``          src/fm_scanner.cpp:1455-1474

Every compute call runs on the GPU through libspeq_scan.so; nothing here computes counts on the CPU.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from ._lib import (SPEQ_MODE_GLOBAL, SPEQ_MODE_LOCAL, BuildOpts, IndexInfo, ScanParams, Slot, SpeqError,  # noqa: F401
                   StreamStats, check, lib)

__all__ = ["FmIndex", "DeviceIndex", "Node", "Pipeline", "ScanResult", "Groupings", "EmHistogram", "Comm", "file_to_map", "unique_to_percent",
           "em_refine", "pack_records", "SpeqError", "SPEQ_MODE_GLOBAL", "SPEQ_MODE_LOCAL"]


def _u64p(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_uint64))


def pack_records(records: Sequence[bytes | str]) -> tuple[bytes, np.ndarray]:
    """Concatenates sequences into one byte buffer + (n+1) u64 offsets."""
    bs = [r.encode() if isinstance(r, str) else bytes(r) for r in records]
    off = np.zeros(len(bs) + 1, dtype=np.uint64)
    if bs:
        off[1:] = np.cumsum([len(b) for b in bs], dtype=np.uint64)
    return b"".join(bs), off


@dataclass
class Groupings:
    names: list[str]
    scaffolds: list[int]
    counts: list[int]
    errors: str


def file_to_map(path: str) -> Groupings:
    """Parses a genome_groupings file exactly as speq::file_to_map does (file_to_map.cpp:20-119)."""
    L = lib()
    h = C.c_void_p()
    check(L.speq_groupings_parse(path.encode(), C.byref(h)))
    try:
        n = L.speq_groupings_n_groups(h)
        names = [L.speq_groupings_name(h, i).decode() for i in range(n)]
        counts = [int(L.speq_groupings_count(h, i)) for i in range(n)]
        m = L.speq_groupings_n_entries(h)
        p = L.speq_groupings_scaffolds(h)
        scaff = [int(p[i]) for i in range(m)] if m else []
        errs = L.speq_groupings_errors(h).decode()
    finally:
        L.speq_groupings_free(h)
    return Groupings(names, scaff, counts, errs)


def unique_to_percent(unique_in_reads, total_in_reads, unique_in_refs, total_in_refs) -> list[float]:
    """P_i = 100 * u_i / T / (U_ref_i / Tot_ref_i) when Tot_ref_i > 0, else 0 (fm_scanner.cpp:1455-1474)."""
    out = []
    for u, ur, tr in zip(unique_in_reads, unique_in_refs, total_in_refs):
        if float(tr) > 0.0:
            pu = float(ur) / float(tr)
            with np.errstate(all="ignore"):
                out.append(float(np.float64(100.0) * np.float64(u) / np.float64(total_in_reads) / np.float64(pu)))
        else:
            out.append(0.0)
    return out


class FmIndex:
    """Immutable FM-index of the grouped reference collection (host side)."""

    def __init__(self, handle: C.c_void_p, header: bytes = b""):
        self._h = handle
        self.header = header

    @classmethod
    def build(cls, records: Sequence[bytes | str], group_of_record: Sequence[int], n_groups: int,
              prefix_q: int = 0, threads: int = 0, pair_steps: bool = False,
              label_table: bool | str = False, gpu_device: Optional[int] = None,
              triple_steps: bool | str = False) -> "FmIndex":
        """label_table: True/False or "auto" (only for collections of >= 4 M symbols).
        gpu_device: build the suffix array and planes on that GPU (None = host SA-IS); identical results."""
        seq, off = pack_records(records)
        grp = np.asarray(group_of_record, dtype=np.int32)
        h = C.c_void_p()
        opts = BuildOpts(prefix_q, threads, int(pair_steps), 2 if label_table == "auto" else int(bool(label_table)),
                         int(gpu_device is not None),
                         gpu_device if gpu_device is not None else 0,
                         2 if triple_steps == "auto" else int(bool(triple_steps)))
        check(lib().speq_index_build(seq, _u64p(off), len(records), grp.ctypes.data_as(C.POINTER(C.c_int32)),
                                     len(grp), n_groups, C.byref(opts), C.byref(h)))
        return cls(h)

    @classmethod
    def load(cls, path: str) -> "FmIndex":
        h, hdr, hl = C.c_void_p(), C.c_void_p(), C.c_uint64()
        check(lib().speq_index_load(path.encode(), C.byref(h), C.byref(hdr), C.byref(hl)))
        header = C.string_at(hdr, hl.value) if hl.value else b""
        lib().speq_free(hdr)
        return cls(h, header)

    def save(self, path: str, header: bytes = b"") -> None:
        check(lib().speq_index_save(self._h, path.encode(), header if header else None, len(header)))

    def info(self) -> IndexInfo:
        info = IndexInfo()
        check(lib().speq_index_get_info(self._h, C.byref(info)))
        return info

    def array(self, name: str, dtype) -> np.ndarray:
        """Copy of a host array of the index (layout: DESIGN.md §3)."""
        p, nb = C.c_void_p(), C.c_uint64()
        check(lib().speq_index_array(self._h, name.encode(), C.byref(p), C.byref(nb)))
        if nb.value == 0:
            return np.zeros(0, dtype=dtype)
        return np.frombuffer(C.string_at(p, nb.value), dtype=dtype).copy()

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().speq_index_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class ScanResult:
    total: int               # T: passing windows
    ambiguous: int           # reads (or pairs) whose counted windows name >= 2 groups
    unique: np.ndarray       # U[g] (u64)
    weights: Optional[np.ndarray]  # W[g] (f64, local mode only)


class DeviceIndex:
    """A replica of an FmIndex in one GPU's HBM."""

    def __init__(self, index: FmIndex, device: int = 0):
        self.index = index
        self.n_groups = index.info().n_groups
        h = C.c_void_p()
        check(lib().speq_device_open(index.handle, device, C.byref(h)))
        self._h = h

    @property
    def handle(self):
        return self._h

    def scan(self, seq: bytes, qual: bytes, offsets: np.ndarray, k: int, phred_cutoff: int = 30,
             paired: bool = False, local: bool = False) -> ScanResult:
        """Scans host reads (staged to HBM in batches)."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(off) - 1
        G = self.n_groups
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if local else None
        p = ScanParams(k, phred_cutoff, int(paired), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        check(lib().speq_scan_reads(self._h, seq, qual, _u64p(off), n, C.byref(p), _u64p(counts),
                                    w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None))
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w)

    def scan_device(self, d_seq: int, d_qual: int, d_offsets: int, n_reads: int, k: int, d_counts: int,
                    d_weights: int = 0, phred_cutoff: int = 30, paired: bool = False, local: bool = False,
                    stream: int = 0) -> None:
        """Hot path on HBM-resident buffers (raw device pointers, e.g. torch tensor.data_ptr()).

        `stream` is a raw hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); 0 = the null stream."""
        p = ScanParams(k, phred_cutoff, int(paired), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        check(lib().speq_scan_reads_device(self._h, d_seq, d_qual, d_offsets, n_reads, C.byref(p), d_counts,
                                           d_weights or None, stream or None))

    AX_STATS_KEYS = ("wave_iters", "lookup_lanes", "run_lanes", "lookup_waves", "run_waves", "run_windows",
                     "deferred", "filter_pass", "p2_probes", "p2_verify", "chunks", "segments", "qual_bytes",
                     "run_tallied", "run_granules", "refills", "busy_1_4", "busy_5_16", "busy_17_32", "busy_33_64",
                     "cyc_refill", "cyc_lookup", "cyc_run", "cyc_phase2", "cyc_total", "p2_passes",
                     "cyc_p2_filter", "p2_rounds", "cyc_ref_pre", "cyc_ref_stage", "cyc_wave_max", "waves",
                     "cyc_gen0", "cyc_gen1", "cyc_gen2", "cyc_gen3", "cyc_gen4")

    def scan_device_stats(self, d_seq: int, d_qual: int, d_offsets: int, n_reads: int, k: int, d_counts: int,
                          d_weights: int = 0, phred_cutoff: int = 30, paired: bool = False,
                          local: bool = False) -> dict:
        """scan_device through the instrumented anchor-and-extend kernel (speq_scan_reads_device_stats, synchronous):
        the same counters, plus the kernel's work counts by kind (keys AX_STATS_KEYS)."""
        p = ScanParams(k, phred_cutoff, int(paired), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        st = np.zeros(len(self.AX_STATS_KEYS), dtype=np.uint64)
        check(lib().speq_scan_reads_device_stats(self._h, d_seq, d_qual, d_offsets, n_reads, C.byref(p), d_counts,
                                                 d_weights or None, _u64p(st)))
        return {key: int(v) for key, v in zip(self.AX_STATS_KEYS, st)}

    def scan_fastq(self, path1: str, path2: Optional[str] = None, k: int = 21, phred_cutoff: int = 30,
                   local: bool = False, threads: int = 4, em: Optional["EmHistogram"] = None):
        """Streams FASTQ(.gz) file(s) through pinned slots to the GPU (speq_scan_fastq). Paired when path2 is given.
        Returns (ScanResult, stats dict)."""
        G = self.n_groups
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if local else None
        p = ScanParams(k, phred_cutoff, int(path2 is not None), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        st = StreamStats()
        check(lib().speq_scan_fastq(self._h, path1.encode(), path2.encode() if path2 else None, C.byref(p),
                                    em._h if em is not None else None, threads, _u64p(counts),
                                    w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None,
                                    C.byref(st)))
        stats = {"records": st.records, "bases": st.bases, "batches": st.batches, "seconds": st.seconds}
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w), stats

    def scan_fastq_shard(self, path1: str, path2: Optional[str], k: int, shard: int, n_shards: int, cut: int = 0,
                         phred_cutoff: int = 30, local: bool = False, threads: int = 4,
                         em: Optional["EmHistogram"] = None):
        """One rank's share of a FASTQ scan (speq_scan_fastq_shard): the blocks b % n_shards == shard of the cut every
        rank makes. cut 1 (parallel cut) raises SpeqError with code SPEQ_E_RETRY when the input does not fit it."""
        G = self.n_groups
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if local else None
        p = ScanParams(k, phred_cutoff, int(path2 is not None), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        st = StreamStats()
        check(lib().speq_scan_fastq_shard(self._h, em._h if em is not None else None, path1.encode(),
                                          path2.encode() if path2 else None, C.byref(p), threads, shard, n_shards,
                                          cut, _u64p(counts),
                                          w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None,
                                          C.byref(st)))
        stats = {"records": st.records, "bases": st.bases, "batches": st.batches, "seconds": st.seconds}
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w), stats

    def count_unique_kmers_per_group_shard(self, k: int, shard: int, n_shards: int):
        """This shard's partial (U_ref, Tot_ref) of the .dat pass (speq_ref_unique_shard)."""
        G = self.n_groups
        u = np.zeros(G, dtype=np.uint64)
        t = np.zeros(G, dtype=np.uint64)
        check(lib().speq_ref_unique_shard(self._h, k, shard, n_shards, _u64p(u), _u64p(t)))
        return u, t

    def count_unique_kmers_per_group(self, k: int) -> tuple[np.ndarray, np.ndarray]:
        """(U_ref[G], Tot_ref[G]) of the reference-uniqueness pass."""
        G = self.n_groups
        u = np.zeros(G, dtype=np.uint64)
        t = np.zeros(G, dtype=np.uint64)
        check(lib().speq_ref_unique(self._h, k, _u64p(u), _u64p(t)))
        return u, t

    def tune(self, **kw) -> None:
        """Launch tuning (blocks_per_cu=..., grid_blocks=...); never changes results."""
        for k, v in kw.items():
            check(lib().speq_device_set_tuning(self._h, k.encode(), int(v)))

    def tuning(self, key: str) -> int:
        v = C.c_int64()
        check(lib().speq_device_get_tuning(self._h, key.encode(), C.byref(v)))
        return v.value

    def prepare(self, k: int) -> dict:
        """Builds the k-mer interval table of k now (speq_device_prepare); returns its size and build time."""
        n, b, ms = C.c_uint64(), C.c_uint64(), C.c_double()
        check(lib().speq_device_prepare(self._h, k, C.byref(n), C.byref(b), C.byref(ms)))
        return {"distinct_kmers": n.value, "table_bytes": b.value, "build_ms": ms.value}

    def timing(self, on: bool) -> None:
        check(lib().speq_timing_enable(self._h, int(on)))

    def timing_read(self) -> tuple[float, int]:
        ms, n = C.c_double(), C.c_uint64()
        check(lib().speq_timing_read(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def close(self):
        if self._h:
            lib().speq_device_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """One communicator of a one-process-per-GPU job (speq_comm_* / speq_allreduce_*): RCCL (ncclAllReduce over
    xGMI) or host sockets when ranks share a GPU.

    Replaces the host `future.get()` sums of per-thread count vectors (/root/reference/src/fm_scanner.cpp:224-233):
    every rank scans its own read shard and one all-reduce sums the G + 2 counters (and the G weights). Either rank 0
    makes the 128-byte RCCL id with `Comm.unique_id()` and hands it to the other ranks out of band (bench.py broadcasts
    it with torch.distributed), or `Comm.connect` runs the rendezvous through a file (as `speq scan` does)."""

    ID_BYTES = 128
    AUTO, RCCL, HOST = 0, 1, 2

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(Comm.ID_BYTES)
        check(lib().speq_comm_unique_id(buf))
        return buf.raw

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != Comm.ID_BYTES:
            raise ValueError("the RCCL unique id is 128 bytes")
        h = C.c_void_p()
        check(lib().speq_comm_init(nranks, rank, C.create_string_buffer(uid, Comm.ID_BYTES), C.byref(h)))
        self._h, self.nranks, self.rank = h, nranks, rank

    @classmethod
    def connect(cls, nranks: int, rank: int, rendezvous: str, device: int = -1, transport: int = 0,
                timeout_s: int = 120) -> "Comm":
        """speq_comm_connect: file rendezvous at `rendezvous`; transport AUTO (RCCL when every rank has its own GPU),
        RCCL or HOST (loopback sockets; device may be -1)."""
        self = cls.__new__(cls)
        h = C.c_void_p()
        check(lib().speq_comm_connect(nranks, rank, device, rendezvous.encode(), transport, timeout_s, C.byref(h)))
        self._h, self.nranks, self.rank = h, nranks, rank
        return self

    @property
    def transport(self) -> int:
        return lib().speq_comm_transport(self._h)

    def allreduce_host(self, buf: np.ndarray, device: int = -1) -> None:
        """In-place sum over the ranks of a host u64 or f64 array (speq_allreduce_host)."""
        if buf.dtype not in (np.uint64, np.float64) or not buf.flags.c_contiguous:
            raise TypeError("allreduce_host takes a contiguous uint64 or float64 array")
        check(lib().speq_allreduce_host(self._h, device, buf.ctypes.data, buf.size, int(buf.dtype == np.float64)))

    def allreduce_u64(self, d_buf: int, count: int, stream: int = 0) -> None:
        """In-place sum of `count` u64 at device pointer d_buf, enqueued on `stream` (raw hipStream_t)."""
        check(lib().speq_allreduce_u64(self._h, d_buf, count, stream or None))

    def allreduce_f64(self, d_buf: int, count: int, stream: int = 0) -> None:
        check(lib().speq_allreduce_f64(self._h, d_buf, count, stream or None))

    def close(self):
        if self._h:
            lib().speq_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Pipeline:
    """Pinned-slot streaming scan (include/speq_scan.h, speq_pipeline_*): fill a slot on the host, submit it, and
    its copy to HBM overlaps the previous slot's kernel."""

    def __init__(self, dev: DeviceIndex, k: int, phred_cutoff: int = 30, paired: bool = False, local: bool = False,
                 slot_bytes: int = 8 << 20, slot_records: int = 1 << 15, n_slots: int = 3,
                 em: Optional["EmHistogram"] = None):
        self.dev, self.local, self.paired = dev, local, paired
        self.n_groups = dev.n_groups
        p = ScanParams(k, phred_cutoff, int(paired), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        h = C.c_void_p()
        check(lib().speq_pipeline_create(dev.handle, C.byref(p), em._h if em is not None else None, slot_bytes,
                                         slot_records, n_slots, C.byref(h)))
        self._h = h

    def put(self, seq: bytes, qual: bytes, offsets: np.ndarray) -> None:
        """Copies whole records into a free slot (growing it if needed) and submits it."""
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = len(off) - 1
        nb = int(off[-1] - off[0])
        s = Slot()
        check(lib().speq_pipeline_acquire(self._h, C.byref(s)))
        try:
            if nb > s.cap_bytes or n > s.cap_records:
                check(lib().speq_pipeline_reserve(self._h, C.byref(s), nb, n))
            base = int(off[0])
            C.memmove(s.seq, bytes(seq[base:base + nb]), nb)
            C.memmove(s.qual, bytes(qual[base:base + nb]), nb)
            rel = (off - off[0]).astype(np.uint64)
            C.memmove(s.offsets, rel.ctypes.data, (n + 1) * 8)
        except BaseException:
            lib().speq_pipeline_submit(self._h, s.slot, 0)
            raise
        check(lib().speq_pipeline_submit(self._h, s.slot, n))

    def finish(self) -> ScanResult:
        G = self.n_groups
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if self.local else None
        check(lib().speq_pipeline_finish(self._h, _u64p(counts),
                                         w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None))
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w)

    def close(self):
        if self._h:
            lib().speq_pipeline_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EmHistogram:
    """{multi-group SA interval -> multiplicity} of the passing windows of a read set (include/speq_scan.h, EM).

    Replaces the reference's re-scan of every read in every EM iteration (fm_scanner.cpp:1069-1453): one GPU scan
    fills the histogram, then every iteration is a host sweep over it (step)."""

    def __init__(self, dev: "DeviceIndex"):
        self.dev = dev
        self.n_groups = dev.n_groups
        h = C.c_void_p()
        check(lib().speq_em_create(dev.index.handle, dev.handle, C.byref(h)))
        self._h = h

    def scan(self, seq: bytes, qual: bytes, offsets: np.ndarray, k: int, phred_cutoff: int = 30,
             paired: bool = False, local: bool = False) -> ScanResult:
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        G = self.n_groups
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if local else None
        p = ScanParams(k, phred_cutoff, int(paired), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        check(lib().speq_em_scan_reads(self._h, seq, qual, _u64p(off), len(off) - 1, C.byref(p), _u64p(counts),
                                       w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None))
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w)

    def allreduce(self, comm: "Comm", stream: int = 0) -> None:
        """Sums the unfinalized histogram over the ranks of comm (speq_em_allreduce)."""
        check(lib().speq_em_allreduce(self._h, comm._h, stream or None))

    def finalize(self, threads: int = 0) -> None:
        check(lib().speq_em_finalize(self._h, threads))

    def info(self) -> tuple[int, int, int]:
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().speq_em_info(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value

    def step(self, percent, group_counts, unique) -> np.ndarray:
        p = np.ascontiguousarray(percent, dtype=np.float64)
        gc = np.ascontiguousarray(group_counts, dtype=np.int32)
        u = np.ascontiguousarray(unique, dtype=np.uint64)
        nxt = np.zeros(self.n_groups, dtype=np.float64)
        dp = C.POINTER(C.c_double)
        check(lib().speq_em_step(self._h, p.ctypes.data_as(dp), gc.ctypes.data_as(C.POINTER(C.c_int32)), _u64p(u),
                                 nxt.ctypes.data_as(dp)))
        return nxt

    def close(self):
        if self._h:
            lib().speq_em_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Node:
    """Replicas of one FmIndex on several GPUs of this process (or logical shards on one GPU): SURVEY.md 8(e).

    Reads shard across the replicas (speq_scan_fastq_multi), the .dat pass splits the reference windows
    (speq_ref_unique_multi), and per-replica EM histograms fold into the first one (speq_em_merge)."""

    def __init__(self, index: FmIndex, devices: Sequence[int]):
        if not devices:
            raise ValueError("Node needs at least one device")
        self.index = index
        self.devices = [DeviceIndex(index, d) for d in devices]
        self.n_groups = self.devices[0].n_groups
        n = len(self.devices)
        self._arr = (C.c_void_p * n)(*[d.handle.value for d in self.devices])

    def __len__(self):
        return len(self.devices)

    def em_histograms(self) -> list["EmHistogram"]:
        return [EmHistogram(d) for d in self.devices]

    def scan_fastq(self, path1: str, path2: Optional[str] = None, k: int = 21, phred_cutoff: int = 30,
                   local: bool = False, threads: int = 4, ems: Optional[Sequence["EmHistogram"]] = None):
        """speq_scan_fastq over every replica; returns (ScanResult, stats dict) of the whole node."""
        G = self.n_groups
        n = len(self.devices)
        counts = np.zeros(G + 2, dtype=np.uint64)
        w = np.zeros(G, dtype=np.float64) if local else None
        p = ScanParams(k, phred_cutoff, int(path2 is not None), SPEQ_MODE_LOCAL if local else SPEQ_MODE_GLOBAL)
        st = StreamStats()
        em_arr = (C.c_void_p * n)(*[e._h.value for e in ems]) if ems is not None else None
        check(lib().speq_scan_fastq_multi(self._arr, em_arr, n, path1.encode(), path2.encode() if path2 else None,
                                          C.byref(p), threads, _u64p(counts),
                                          w.ctypes.data_as(C.POINTER(C.c_double)) if w is not None else None,
                                          C.byref(st)))
        stats = {"records": st.records, "bases": st.bases, "batches": st.batches, "seconds": st.seconds}
        return ScanResult(int(counts[0]), int(counts[1]), counts[2:].copy(), w), stats

    def count_unique_kmers_per_group(self, k: int) -> tuple[np.ndarray, np.ndarray]:
        G = self.n_groups
        u = np.zeros(G, dtype=np.uint64)
        t = np.zeros(G, dtype=np.uint64)
        check(lib().speq_ref_unique_multi(self._arr, len(self.devices), k, _u64p(u), _u64p(t)))
        return u, t

    @staticmethod
    def merge_em(ems: Sequence["EmHistogram"]) -> "EmHistogram":
        """Folds ems[1:] into ems[0] (which is returned; the others accept only close())."""
        for e in ems[1:]:
            check(lib().speq_em_merge(ems[0]._h, e._h))
        return ems[0]

    def close(self):
        for d in self.devices:
            d.close()


def em_refine(step, unique_totals, total, percent0, precision: float = 1e-6, max_iterations: int = 1000):
    """The reference's refinement loop (fm_scanner.cpp:248-279): starting from diff = 1.0 per group, while
    max(diff) > precision: next_tkpg = step(percent); percent' = unique_to_percent(unique_totals, total,
    unique_totals, next_tkpg); diff = |percent' - percent|. Returns [(percent', next_tkpg), ...] per iteration."""
    percent = list(percent0)
    out = []
    diff = [1.0] * len(percent)
    while _max_element(diff) > precision and len(out) < max_iterations:
        nxt = step(np.asarray(percent, dtype=np.float64))
        new = unique_to_percent(unique_totals, total, unique_totals, nxt)
        diff = [abs(x - y) for x, y in zip(new, percent)]
        percent = new
        out.append((list(new), [float(x) for x in nxt]))
    return out


def _max_element(v):
    """std::max_element with operator< (NaN never compares greater, so a leading NaN wins)."""
    best = v[0]
    for x in v[1:]:
        if best < x:
            best = x
    return best
