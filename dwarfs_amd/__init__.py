"""dwarfs_amd -- MI355X-native ricepp block codec for DwarFS.

The hot path of mhx/dwarfs's `fits/image` category (ricepp encode/decode of
independent 16-bit sample blocks) as hand-written HIP kernels for gfx950,
reached through the C ABI of include/ricepp_amd.h.
"""

from .codec import (  # noqa: F401
    CodecConfig,
    Decoder,
    Encoder,
    EncodedBatch,
    OutOfRange,
    UnsupportedConfiguration,
    create_decoder,
    create_encoder,
    decode_batch,
    encode_batch,
    worst_case_encoded_bytes,
)
