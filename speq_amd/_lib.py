"""ctypes binding of libspeq_scan.so (include/speq_scan.h).

The product path is the HIP library: if the shared object is missing this module raises at import time
instead of falling back to anything on the CPU.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# SPEQ_LIB_PATH selects an alternative build of the same library (A/B kernel variants in scripts/).
LIB_PATH = os.environ.get("SPEQ_LIB_PATH") or os.path.join(_HERE, "libspeq_scan.so")


class SpeqError(RuntimeError):
    """A non-zero status from the C ABI; .code is the SPEQ_E_* value."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"speq error {code}: {msg}")
        self.code = code


SPEQ_OK, SPEQ_E_ARG, SPEQ_E_IO, SPEQ_E_DEVICE, SPEQ_E_GROUPS, SPEQ_E_NOMEM, SPEQ_E_RETRY = 0, -1, -2, -3, -4, -5, -6
SPEQ_MODE_GLOBAL, SPEQ_MODE_LOCAL = 0, 1


class BuildOpts(C.Structure):
    _fields_ = [("prefix_q", C.c_uint32), ("threads", C.c_uint32), ("pair_steps", C.c_uint32),
                ("label_table", C.c_uint32), ("gpu_build", C.c_uint32), ("device", C.c_int32),
                ("triple_steps", C.c_uint32)]


class ScanParams(C.Structure):
    _fields_ = [("k", C.c_uint32), ("phred_cutoff", C.c_uint32), ("paired", C.c_uint32), ("mode", C.c_uint32)]


class IndexInfo(C.Structure):
    _fields_ = [("n", C.c_uint64), ("n_texts", C.c_uint32), ("n_records", C.c_uint32), ("n_groups", C.c_uint32),
                ("prefix_q", C.c_uint32), ("pair_steps", C.c_uint32), ("label_table", C.c_uint32),
                ("n_runs", C.c_uint64),
                ("device_bytes", C.c_uint64), ("triple_steps", C.c_uint32)]


# name -> (restype, argtypes); every symbol declared in include/speq_scan.h
_P, _U8P, _U64P, _I32P, _F64P = C.c_void_p, C.POINTER(C.c_uint8), C.POINTER(C.c_uint64), C.POINTER(C.c_int32), \
    C.POINTER(C.c_double)
class Slot(C.Structure):
    _fields_ = [("seq", C.POINTER(C.c_uint8)), ("qual", C.POINTER(C.c_uint8)), ("offsets", C.POINTER(C.c_uint64)),
                ("cap_bytes", C.c_uint64), ("cap_records", C.c_uint64), ("slot", C.c_int32)]


class StreamStats(C.Structure):
    _fields_ = [("records", C.c_uint64), ("bases", C.c_uint64), ("batches", C.c_uint64), ("seconds", C.c_double)]


SIGNATURES = {
    "speq_last_error": (C.c_char_p, []),
    "speq_abi_version": (C.c_int, []),
    "speq_device_count": (C.c_int, []),
    "speq_index_build": (C.c_int, [C.c_char_p, _U64P, C.c_uint32, _I32P, C.c_uint32, C.c_uint32,
                                   C.POINTER(BuildOpts), C.POINTER(_P)]),
    "speq_index_save": (C.c_int, [_P, C.c_char_p, _P, C.c_uint64]),
    "speq_index_load": (C.c_int, [C.c_char_p, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_uint64)]),
    "speq_index_read_header": (C.c_int, [C.c_char_p, C.POINTER(_P), C.POINTER(C.c_uint64)]),
    "speq_index_free": (None, [_P]),
    "speq_free": (None, [_P]),
    "speq_index_get_info": (C.c_int, [_P, C.POINTER(IndexInfo)]),
    "speq_index_array": (C.c_int, [_P, C.c_char_p, C.POINTER(_P), C.POINTER(C.c_uint64)]),
    "speq_device_warmup": (C.c_int, [C.c_int, C.c_uint32]),
    "speq_stream_reserve": (C.c_int, [C.c_int, C.c_uint32, C.c_uint32]),
    "speq_device_open": (C.c_int, [_P, C.c_int, C.POINTER(_P)]),
    "speq_device_close": (C.c_int, [_P]),
    "speq_scan_reads_device": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.POINTER(ScanParams), _P, _P, _P]),
    "speq_scan_reads_device_stats": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.POINTER(ScanParams), _P, _P, _U64P]),
    "speq_scan_reads": (C.c_int, [_P, C.c_char_p, C.c_char_p, _U64P, C.c_uint64, C.POINTER(ScanParams),
                                  _U64P, _F64P]),
    "speq_ref_unique": (C.c_int, [_P, C.c_uint32, _U64P, _U64P]),
    "speq_ref_unique_device": (C.c_int, [_P, C.c_uint32, _P, _P, _P]),
    "speq_comm_unique_id": (C.c_int, [_P]),
    "speq_comm_init": (C.c_int, [C.c_int, C.c_int, _P, C.POINTER(_P)]),
    "speq_comm_connect": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_int, C.c_int, C.POINTER(_P)]),
    "speq_comm_transport": (C.c_int, [_P]),
    "speq_comm_destroy": (C.c_int, [_P]),
    "speq_allreduce_u64": (C.c_int, [_P, _P, C.c_uint64, _P]),
    "speq_allreduce_f64": (C.c_int, [_P, _P, C.c_uint64, _P]),
    "speq_em_create": (C.c_int, [_P, _P, C.POINTER(_P)]),
    "speq_em_scan_reads": (C.c_int, [_P, C.c_char_p, C.c_char_p, _U64P, C.c_uint64, C.POINTER(ScanParams),
                                     _U64P, _F64P]),
    "speq_em_scan_reads_device": (C.c_int, [_P, _P, _P, _P, C.c_uint64, C.POINTER(ScanParams), _P, _P, _P]),
    "speq_em_finalize": (C.c_int, [_P, C.c_uint32]),
    "speq_em_info": (C.c_int, [_P, _U64P, _U64P, _U64P]),
    "speq_em_step": (C.c_int, [_P, _F64P, _I32P, _U64P, _F64P]),
    "speq_em_free": (None, [_P]),
    "speq_pipeline_create": (C.c_int, [_P, C.POINTER(ScanParams), _P, C.c_uint64, C.c_uint64, C.c_uint32,
                                       C.POINTER(_P)]),
    "speq_pipeline_acquire": (C.c_int, [_P, C.POINTER(Slot)]),
    "speq_pipeline_reserve": (C.c_int, [_P, C.POINTER(Slot), C.c_uint64, C.c_uint64]),
    "speq_pipeline_submit": (C.c_int, [_P, C.c_int32, C.c_uint64]),
    "speq_pipeline_finish": (C.c_int, [_P, _U64P, _F64P]),
    "speq_pipeline_free": (None, [_P]),
    "speq_scan_fastq": (C.c_int, [_P, C.c_char_p, C.c_char_p, C.POINTER(ScanParams), _P, C.c_uint32, _U64P, _F64P,
                                  C.POINTER(StreamStats)]),
    "speq_scan_fastq_multi": (C.c_int, [C.POINTER(_P), C.POINTER(_P), C.c_uint32, C.c_char_p, C.c_char_p,
                                        C.POINTER(ScanParams), C.c_uint32, _U64P, _F64P, C.POINTER(StreamStats)]),
    "speq_ref_unique_multi": (C.c_int, [C.POINTER(_P), C.c_uint32, C.c_uint32, _U64P, _U64P]),
    "speq_em_merge": (C.c_int, [_P, _P]),
    "speq_fastq_checksum": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint32, _U64P, _U64P, _U64P]),
    "speq_scan_fastq_shard": (C.c_int, [_P, _P, C.c_char_p, C.c_char_p, C.POINTER(ScanParams), C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_int, _U64P, _F64P, C.POINTER(StreamStats)]),
    "speq_fastq_checksum_shard": (C.c_int, [C.c_char_p, C.c_char_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int,
                                            _U64P, _U64P, _U64P]),
    "speq_ref_unique_shard": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, _U64P, _U64P]),
    "speq_em_allreduce": (C.c_int, [_P, _P, _P]),
    "speq_allreduce_host": (C.c_int, [_P, C.c_int, _P, C.c_uint64, C.c_int]),
    "speq_groupings_parse": (C.c_int, [C.c_char_p, C.POINTER(_P)]),
    "speq_groupings_n_groups": (C.c_uint32, [_P]),
    "speq_groupings_name": (C.c_char_p, [_P, C.c_uint32]),
    "speq_groupings_count": (C.c_int32, [_P, C.c_uint32]),
    "speq_groupings_n_entries": (C.c_uint32, [_P]),
    "speq_groupings_scaffolds": (_I32P, [_P]),
    "speq_groupings_errors": (C.c_char_p, [_P]),
    "speq_groupings_free": (None, [_P]),
    "speq_device_set_tuning": (C.c_int, [_P, C.c_char_p, C.c_int64]),
    "speq_device_get_tuning": (C.c_int, [_P, C.c_char_p, C.POINTER(C.c_int64)]),
    "speq_device_prepare": (C.c_int, [_P, C.c_uint32, _U64P, _U64P, _F64P]),
    "speq_timing_enable": (C.c_int, [_P, C.c_int]),
    "speq_timing_read": (C.c_int, [_P, _F64P, _U64P]),
}

_lib = None
ABI_VERSION = 7  # include/speq_scan.h SPEQ_ABI_VERSION (struct layouts above)


def lib() -> C.CDLL:
    """Loads libspeq_scan.so (raises loudly when it has not been built).

    A process that also uses torch must import torch BEFORE the first call: torch links its bundled HIP runtime
    by the unversioned name, so loading ours first would leave two HIP runtimes in the process."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build()); "
                              "the SPeQ scan path has no CPU fallback")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.speq_abi_version() != ABI_VERSION:
            raise ImportError(f"{LIB_PATH} has ABI {L.speq_abi_version()}, this binding expects {ABI_VERSION}: "
                              "rebuild with `make`")
        _lib = L
    return _lib


def check(rc: int) -> None:
    if rc != SPEQ_OK:
        raise SpeqError(rc, lib().speq_last_error().decode(errors="replace"))
