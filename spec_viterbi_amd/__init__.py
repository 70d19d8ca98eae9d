"""spec_viterbi_amd -- MI355X (gfx950) engine for Viterbi as (min,+) linear algebra.

Drop-in backend for IvanTyulyandin/Spec_Viterbi's hot path (per-observation (min,+) step,
emission masking, precomputed _spec products).  See DESIGN.md / INTEGRATION.md.
"""
from .hmm import HMM, ZERO_PROB, almost_equal, pack_sequences, read_emit_seq, read_HMM, to_modified_prob
from .stream import SeqReader, decode_file, read_sequences
from .viterbi import (DeviceBatch, DeviceModel, HIP_impl, HIP_spec_impl, Viterbi_impl, Viterbi_spec_impl,
                      pinned_empty)

__all__ = [
    "HMM", "ZERO_PROB", "almost_equal", "to_modified_prob", "read_HMM", "read_emit_seq", "pack_sequences",
    "DeviceModel", "DeviceBatch", "Viterbi_impl", "Viterbi_spec_impl", "HIP_impl", "HIP_spec_impl",
    "SeqReader", "read_sequences", "decode_file", "pinned_empty",
]
