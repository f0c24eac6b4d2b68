"""panman_amd -- MI355X-native Fitch/Sankoff small parsimony for PanMAN (HIP, gfx950).

The compute path is libpanman_amd.so (hand-written HIP kernels behind the C-ABI in
include/panman_gpu.h); this package is its host-side binding.  No CPU fallback exists.
"""
from ._lib import LIB_PATH, build_id, MODE_BLOCK_FITCH, MODE_BLOCK_SANKOFF, MODE_FITCH, MODE_SANKOFF, PanmanError, header_symbols, load, phase_report, phase_reset  # noqa: F401
from .engine import Engine, fasta_multi, msa_build, msa_to_panman, pack_codes, random_join_tree, sars_like_tree, stream_copy_rate, stream_write_rate  # noqa: F401
from .engine import chunk_entries, chunk_pack, chunk_unpack, comm_unique_id, multi_run, shard_range_c  # noqa: F401
from .panmat import PanMAT, PanmanFile, write_panman  # noqa: F401,E402
