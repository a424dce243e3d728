"""spark-bam on MI355X: host-side mirror of spark-bam's BGZF + record-boundary API over
the C-ABI in include/sparkbam.h (libsparkbam_hip.so, hand-written gfx950 kernels).

Import name: ``spark_bam_amd`` (the directory name contains a hyphen, so load it with
``__graft_entry__.load_package()`` or importlib).  Names follow the reference:

  bgzf:   Pos, Header.make, Metadata, FindBlockStart, Stream (blocks / inflated bytes)
  check:  eager.Checker / full.Checker (batched over positions; per-position windowed
          WindowedEagerChecker / WindowedFullChecker), FindRecordStart
  load:   load_splits_and_reads / load_bam_count / load_reads / load_bam_intervals
          (CanLoadBam), FileSplits, read_bai (bam.index.Index)
"""
from ._lib import (BLOCK_EMPTY, BLOCK_TRUNCATED, FULL_FLAGS_MASK, FULL_N_SHIFT,  # noqa: F401
                   FULL_SUCCESS, FULL_UNKNOWN, HeaderParseException, HeaderSearchFailedException,
                   NoReadFoundException, SparkBamError, lib)
from .device import Context, PinnedBuffer, Shard  # noqa: F401
from .api import (FLAG_NAMES, htsjdk_rewrite, Header, Metadata, Pos, Split, bam_header, check_bam,  # noqa: F401
                  file_splits, full_check, load_bam_count, load_reads, load_splits_and_reads,
                  parse_bam_header)
from .records import Reads  # noqa: F401
from .checkers import GpuWindow, WindowedEagerChecker, WindowedFullChecker  # noqa: F401
from .intervals import (Chunk, Index, get_interval_chunks, load_bam_intervals,  # noqa: F401
                        parse_loci, read_bai)

__all__ = [
    "htsjdk_rewrite",
    "Context", "PinnedBuffer", "Shard", "SparkBamError", "HeaderParseException", "HeaderSearchFailedException",
    "NoReadFoundException", "Pos", "Header", "Metadata", "Split", "FLAG_NAMES",
    "file_splits", "load_splits_and_reads", "load_bam_count", "check_bam", "full_check",
    "bam_header", "parse_bam_header", "lib", "load_reads", "Reads", "Chunk", "Index",
    "read_bai", "parse_loci", "get_interval_chunks", "load_bam_intervals",
    "GpuWindow", "WindowedEagerChecker", "WindowedFullChecker",
]
