"""speq_amd — MI355X-native SPeQ scan path.

A from-scratch FM-index laid out in HBM, a hand-written CDNA4 (gfx950) HIP backward-search kernel that tallies
k-mers unique to one variant, and one RCCL all-reduce of the per-variant counters. The reference is
ibharvey/speq (C++/SeqAn3); see DESIGN.md for the path, the boundary and the data layout.
"""
from ._lib import SpeqError, lib  # noqa: F401  (raises if libspeq_scan.so is missing)
from .api import (SPEQ_MODE_GLOBAL, SPEQ_MODE_LOCAL, Comm, DeviceIndex, EmHistogram, FmIndex, Groupings, Node, Pipeline,  # noqa: F401,E501
                  ScanResult, em_refine, file_to_map, pack_records, unique_to_percent)

__version__ = "0.1.0"
