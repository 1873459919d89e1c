/*
 * ricepp_amd.h -- C ABI of the MI355X-native ricepp block codec.
 *
 * This is the drop-in boundary: plain C types, device pointers and sizes, no
 * torch or C++ types.  It replaces the inner ricepp library API that the
 * DwarFS plugin binds (reference: /root/reference):
 *
 *   rpp_check_config      <- ricepp::create_encoder / create_decoder config
 *                            validation (ricepp/ricepp_cpuspecific_traits.h:118-151,
 *                            throws at ricepp/ricepp_cpuspecific.cpp:161,173)
 *   rpp_worst_case_bytes  <- encoder_interface::worst_case_encoded_bytes
 *                            (ricepp/include/ricepp/encoder_interface.h:38-60,
 *                            ricepp/ricepp_cpuspecific.cpp:58-66,75-77,
 *                            ricepp/include/ricepp/codec.h:142-151)
 *   rpp_encode_batch /    <- encoder_interface::encode(span<u8>, span<u16 const>)
 *   rpp_encode_batch_ws
 *                            (ricepp/ricepp_cpuspecific.cpp:68-72,101-108), one
 *                            call per DwarFS block in src/compression/ricepp.cpp:136-137,
 *                            batched over many independent blocks
 *   rpp_decode_batch /    <- decoder_interface::decode(span<u16>, span<u8 const>)
 *   rpp_decode_batch_ws
 *                            (ricepp/include/ricepp/decoder_interface.h:37-50,
 *                            ricepp/ricepp_cpuspecific.cpp:127-144), called by
 *                            src/compression/ricepp.cpp:215-232
 *   rpp_unused_lsb_batch  <- the FITS categorizer's unused-LSB detection
 *                            (src/writer/categorizer/fits_categorizer.cpp:118-178),
 *                            which picks the codec's unused_lsb_count
 *   rpp_exclusive_scan_u64 <- the writer's running image offset as it appends
 *   rpp_pack_batch           compressed blocks (src/writer/filesystem_writer.cpp:255-287)
 *   rpp_pcm_unpack /      <- pcm_sample_transformer<int32_t>::unpack / pack
 *   rpp_pcm_pack             (include/dwarfs/pcm_sample_transformer.h:40-71,
 *                            src/pcm_sample_transformer.cpp:44-228), the PCM
 *                            front end of the FLAC compressor (src/compression/flac.cpp:211,322)
 *   rpp_frame_header /    <- the DwarFS block framing of src/compression/ricepp.cpp:
 *   rpp_parse_frame          varint size + thrift-compact ricepp_block_header
 *                            (:107-127 write, :186-201,237-249 read)
 *
 * Errors: C++ exceptions cannot cross this boundary.  Status codes map back to
 * the reference's exceptions in the C++ facade (include/ricepp_amd.hpp):
 *   RPP_UNSUPPORTED_CONFIG -> std::runtime_error("Unsupported configuration")
 *   RPP_TRUNCATED_INPUT    -> std::out_of_range (bitstream_reader.h:150-152)
 *
 * Memory: every pointer passed to the *_batch calls is DEVICE memory owned by
 * the caller (hipMalloc'd).  Calls are asynchronous on `stream` (a
 * hipStream_t; NULL = default stream), which must belong to the current
 * device (rpp_decode_batch_ws / _ex return RPP_INVALID_ARGUMENT otherwise).
 * Per-block status / sizes are written to device arrays and are valid once
 * the stream has been synchronised.
 */
#ifndef RICEPP_AMD_H
#define RICEPP_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RPP_OK 0
#define RPP_UNSUPPORTED_CONFIG (-1)
#define RPP_TRUNCATED_INPUT (-2)
#define RPP_INVALID_ARGUMENT (-3)
#define RPP_OUTPUT_TOO_SMALL (-4)
#define RPP_HIP_ERROR (-5)
/* A device-side consistency bound tripped (a decode tile waited longer than
 * its bound for a predecessor's prefix): the block's output is invalid.  Never
 * returned for well-formed or malformed input; it reports a bug or a stalled
 * GPU instead of returning wrong samples as RPP_OK. */
#define RPP_INTERNAL_ERROR (-6)

/* ricepp::codec_config (ricepp/include/ricepp/codec_config.h:36-41). */
typedef struct rpp_config {
  uint32_t block_size;             /* ricepp sub-block size, 1..512 */
  uint32_t component_stream_count; /* 1 or 2 */
  uint32_t big_endian;             /* stored sample byte order: 1 = big */
  uint32_t unused_lsb_count;       /* 0..15 */
} rpp_config;

/* Streams hold fewer samples than this: mkdwarfs blocks go up to 2^30 bytes
 * (-S 30, tools/src/mkdwarfs_main.cpp:135), i.e. 2^29 samples.  Streams of
 * 2^27 samples and more are encoded in segments by rpp_encode_batch_ws (the
 * workspace-free rpp_encode_batch, one wave per stream, takes fewer) and
 * decoded one wave each (not segmented). */
#define RPP_MAX_STREAM_SAMPLES (UINT64_C(1) << 30)

/* ABI version, bumped on any signature change. */
uint32_t rpp_abi_version(void);

/* RPP_OK or RPP_UNSUPPORTED_CONFIG. */
int rpp_check_config(const rpp_config* cfg);

/* ceil(cs * (16 + 4*ceil((n/cs)/bs) + 16*(n/cs)) / 8) bytes. */
uint64_t rpp_worst_case_bytes(const rpp_config* cfg, uint64_t n_samples);

/*
 * Encode `nblocks` independent ricepp streams.
 *   d_in          stored uint16 samples
 *   d_in_offsets  [nblocks] start of block b in d_in, in samples, 8-aligned
 *   d_n_samples   [nblocks] samples in block b (multiple of cs, < RPP_MAX_STREAM_SAMPLES)
 *   d_out         output bytes
 *   d_out_offsets [nblocks] byte offset of block b's output, 16-aligned;
 *                 the region must hold rpp_worst_case_bytes(n_samples[b])
 *   d_out_bytes   [nblocks] written: encoded size of block b
 *   d_status      [nblocks] written: RPP_OK or an error code
 * Returns RPP_OK if the launch was issued, else an error code.
 */
int rpp_encode_batch(const rpp_config* cfg, const uint16_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_n_samples, uint32_t nblocks, uint8_t* d_out,
                     const uint64_t* d_out_offsets, uint64_t* d_out_bytes, int32_t* d_status,
                     void* stream);

/*
 * Device workspace rpp_encode_batch_ws needs for `nblocks` streams holding
 * `total_samples` samples in all, none longer than `max_stream_samples`
 * (0: no workspace needed; also for an unsupported config).
 */
uint64_t rpp_encode_workspace_bytes(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                    uint32_t nblocks);

/*
 * rpp_encode_batch with a caller-owned device workspace of at least
 * rpp_encode_workspace_bytes(cfg, total_samples, max_stream_samples, nblocks)
 * bytes (total_samples >= the sum and max_stream_samples >= the maximum of
 * d_n_samples).  Streams longer than 256 chunks of cs * bs samples are encoded
 * by several waves in parallel (a segment per 256 chunks, then the segments'
 * bits are placed at their offsets), so a 16 MiB DwarFS block no longer
 * encodes at one wave's speed; a batch without such streams is exactly
 * rpp_encode_batch.  Same output as rpp_encode_batch, byte for byte.  Fully
 * asynchronous on `stream`.
 */
int rpp_encode_batch_ws(const rpp_config* cfg, const uint16_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_n_samples, uint32_t nblocks, uint8_t* d_out,
                        const uint64_t* d_out_offsets, uint64_t* d_out_bytes, int32_t* d_status,
                        uint64_t total_samples, uint64_t max_stream_samples, void* d_workspace,
                        uint64_t workspace_bytes, void* stream);

/*
 * Decode `nblocks` independent ricepp streams.
 *   d_in          encoded bytes
 *   d_in_offsets  [nblocks] byte offset of block b's stream (any alignment: a
 *                 DwarFS payload right after its varint + thrift header)
 *   d_in_bytes    [nblocks] encoded size of block b
 *   d_out         decoded stored uint16 samples
 *   d_out_offsets [nblocks] start of block b's output, in samples, 8-aligned
 *   d_n_samples   [nblocks] samples to decode (multiple of cs)
 *   d_status      [nblocks] RPP_OK, RPP_TRUNCATED_INPUT (the reference's
 *                 std::out_of_range) or RPP_INVALID_ARGUMENT
 * This workspace-free form ALWAYS decodes one stream per wavefront (parse
 * and values fused; bs 16 / 32: four streams per wavefront, one per 16-lane
 * row, any stream that path leaves then one per wavefront), fully
 * asynchronously on `stream`.  That is the fast
 * path for batches of many short streams (thousands of 64 KiB blocks), but a
 * long stream then decodes at one wave's speed (a 16 MiB block: ~30 ms).
 * Batches with long streams should use rpp_decode_batch_ws, which splits
 * them over many waves.
 */
int rpp_decode_batch(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                     const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out,
                     const uint64_t* d_out_offsets, const uint64_t* d_n_samples,
                     int32_t* d_status, void* stream);

/*
 * Device workspace rpp_decode_batch_ws needs for a batch of `nblocks` streams
 * holding `total_samples` samples in all, the longest `max_stream_samples`
 * (0: none needed, or an unsupported config).
 */
uint64_t rpp_decode_workspace_bytes(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                    uint32_t nblocks);

/*
 * rpp_decode_batch with the batch's sample counts and a caller-owned device
 * workspace of at least rpp_decode_workspace_bytes(cfg, total_samples,
 * max_stream_samples, nblocks) bytes, where total_samples >= the sum of
 * d_n_samples and max_stream_samples >= the largest.  Fully asynchronous on
 * `stream` (graph-capturable: no host synchronisation; a segmented call forks
 * part of its work onto a side stream private to `stream` and joins it before
 * returning).  A batch whose longest stream holds more than 1/1024 of its
 * samples (and >= 2^18) is decoded segmented: long streams are cut into units
 * of 2^18..2^23 bits parsed by one wave each from a guessed first header,
 * stitched exactly, then every sub-block of every stream is decoded by its
 * own lane; other batches one wave per stream.  If the device finds the
 * batch larger than total_samples / max_stream_samples promised, it decodes
 * the whole batch one wave per stream instead (correct, never out of the
 * workspace's bounds).
 */
int rpp_decode_batch_ws(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out,
                        const uint64_t* d_out_offsets, const uint64_t* d_n_samples, int32_t* d_status,
                        uint64_t total_samples, uint64_t max_stream_samples, void* d_workspace,
                        uint64_t workspace_bytes, void* stream);

/*
 * Explicit decode path selection (tests, diagnostics, tuning).  A NULL
 * options pointer or a zeroed struct is exactly rpp_decode_batch_ws.
 */
#define RPP_DECODE_AUTO 0      /* segmented when the batch has long streams */
#define RPP_DECODE_FUSED 1     /* one wave per stream, never segmented */
#define RPP_DECODE_SEGMENTED 2 /* every stream longer than one unit is split */
/* test_flags: fault injection and diagnostics, 0 in production */
#define RPP_TEST_NO_FAST_LANES 1u   /* extraction: every lane takes the general path */
#define RPP_TEST_LOOKBACK_STALL 2u  /* extraction: tile 1 of each stream never publishes its prefix,
                                       and the look-back gives up after 2^10 polls (-> RPP_INTERNAL_ERROR) */
#define RPP_TEST_PHASE_TIMERS 4u    /* extraction: per-phase cycle counters (diagnostic builds' tools) */
typedef struct rpp_decode_options {
  uint32_t path;        /* RPP_DECODE_AUTO / _FUSED / _SEGMENTED */
  uint32_t seg_log2;    /* units of 2^seg_log2 bits, 10..26; 0: chosen from the batch */
  uint32_t fused_waves; /* streams per workgroup of the one-wave-per-stream kernel, 1..16; 0: auto */
  uint32_t test_flags;  /* RPP_TEST_* */
} rpp_decode_options;

uint64_t rpp_decode_workspace_bytes_ex(const rpp_config* cfg, uint64_t total_samples, uint64_t max_stream_samples,
                                       uint32_t nblocks, const rpp_decode_options* opt);
int rpp_decode_batch_ex(const rpp_config* cfg, const uint8_t* d_in, const uint64_t* d_in_offsets,
                        const uint64_t* d_in_bytes, uint32_t nblocks, uint16_t* d_out,
                        const uint64_t* d_out_offsets, const uint64_t* d_n_samples, int32_t* d_status,
                        uint64_t total_samples, uint64_t max_stream_samples, void* d_workspace,
                        uint64_t workspace_bytes, const rpp_decode_options* opt, void* stream);

/*
 * Unused least-significant bits of 16-bit images (the FITS categorizer's
 * get_unused_lsb_count, src/writer/categorizer/fits_categorizer.cpp:118-178):
 * for each image, the OR of all its samples (converted from big endian when
 * big_endian != 0) and d_counts[i] = its number of trailing zero bits
 * (std::countr_zero of a uint16_t: 16 for an all-zero or empty image).
 *   d_in          stored uint16 samples
 *   d_offsets     [nimages] first sample of image i
 *   d_n_samples   [nimages] samples of image i, each <= max_samples
 *   d_work        [nimages] device scratch (overwritten)
 *   d_counts      [nimages] written: unused LSB count of image i
 * Asynchronous on `stream`; nimages <= 65535 per call.
 */
int rpp_unused_lsb_batch(const uint16_t* d_in, const uint64_t* d_offsets, const uint64_t* d_n_samples,
                         uint64_t max_samples, uint32_t nimages, uint32_t big_endian, uint32_t* d_work,
                         uint32_t* d_counts, void* stream);

/*
 * Image offsets of a batch of compressed blocks: d_out[b] = sum of d_in[0..b-1]
 * (exclusive prefix sum, uint64).  The DwarFS writer appends compressed blocks
 * back to back (src/writer/filesystem_writer.cpp:255-287); with the encoded
 * sizes of a GPU batch in device memory (all-gathered across ranks) this gives
 * every block's position in the image without a host round trip.
 * d_in may equal d_out only if n <= 1.  Asynchronous on `stream`.
 */
int rpp_exclusive_scan_u64(const uint64_t* d_in, uint64_t n, uint64_t* d_out, void* stream);

/*
 * Pack the encoded streams of a batch (e.g. rpp_encode_batch output, block b at
 * d_src + d_src_offsets[b], 16-aligned, d_sizes[b] bytes) back to back at
 * 16-byte-aligned offsets: d_dst_offsets[b] = sum of round_up(d_sizes[j], 16)
 * for j < b, block b's bytes copied to d_dst + d_dst_offsets[b], *d_total =
 * the packed length.  d_dst must hold sum(round_up(sizes, 16)) bytes (at most
 * the sum of the encode capacities); the source slots must be readable up to
 * round_up(size, 16).  Then one device->host copy of *d_total bytes moves the
 * batch, instead of its worst-case capacity (the writer's block hand-off,
 * src/writer/filesystem_writer.cpp:255-287).  Asynchronous on `stream`.
 */
int rpp_pack_batch(const uint8_t* d_src, const uint64_t* d_src_offsets, const uint64_t* d_sizes, uint32_t nblocks,
                   uint8_t* d_dst, uint64_t* d_dst_offsets, uint64_t* d_total, void* stream);

/*
 * DwarFS ricepp block framing (host memory).  rpp_frame_header writes
 * varint(uncompressed_bytes) + the thrift-compact ricepp_block_header
 * (thrift/compression.thrift:42-49) to `out` (>= 32 bytes) and returns its
 * length.  rpp_parse_frame parses the same, returns the header length or a
 * negative status.
 */
typedef struct rpp_frame {
  uint64_t uncompressed_bytes;
  uint32_t block_size;
  uint32_t component_count;
  uint32_t bytes_per_sample;
  uint32_t unused_lsb_count;
  uint32_t big_endian;
  uint32_t ricepp_version;
} rpp_frame;

size_t rpp_frame_header(const rpp_frame* f, uint8_t* out);
long rpp_parse_frame(const uint8_t* in, size_t in_len, rpp_frame* f);

/*
 * PCM sample format (pcm_sample_transformer's constructor arguments,
 * include/dwarfs/pcm_sample_transformer.h:36-45): bytes per sample 1..4,
 * significant bits 1..8*bytes, big_endian / is_signed / lsb_padded as 0/1.
 * rpp_pcm_check_format: RPP_OK; RPP_UNSUPPORTED_CONFIG for bytes outside 1..4
 * (the reference's runtime_error "unsupported number of bytes per sample: N",
 * src/pcm_sample_transformer.cpp:310-311); RPP_INVALID_ARGUMENT for bits
 * outside 1..8*bytes (asserted by the reference, :354).
 */
typedef struct rpp_pcm_format {
  uint32_t big_endian;
  uint32_t is_signed;
  uint32_t lsb_padded;
  uint32_t bytes;
  uint32_t bits;
} rpp_pcm_format;

int rpp_pcm_check_format(const rpp_pcm_format* f);

/*
 * n_samples PCM samples of `bytes` bytes each at d_src -> int32 at d_dst
 * (pcm_sample_transformer<int32_t>::unpack), and the inverse
 * (pcm_sample_transformer<int32_t>::pack).  Device memory; asynchronous on
 * `stream`.  Any alignment is accepted (4-byte packed / 16-byte int32 buffers
 * take the vector path).
 */
int rpp_pcm_unpack(const rpp_pcm_format* f, const uint8_t* d_src, int32_t* d_dst, uint64_t n_samples, void* stream);
int rpp_pcm_pack(const rpp_pcm_format* f, const int32_t* d_src, uint8_t* d_dst, uint64_t n_samples, void* stream);

/*
 * FLAC blocks (src/compression/flac.cpp).  Parity unpinned: the reference
 * codes them with libFLAC (absent here; no FLAC fixture in the reference).
 *
 * Framing, host side: varint(uncompressed bytes) + thrift-compact
 * flac_block_header (thrift/compression.thrift:36-40; written by
 * flac_block_compressor::compress, flac.cpp:284-304, parsed by
 * flac_block_decompressor, :477-484) + a native FLAC stream.  flags: bit 7
 * big endian, bit 6 signed, bit 5 LSB padding, bits 0-1 bytes per sample - 1
 * (flac.cpp:41-44).  rpp_flac_stream_header writes "fLaC" + STREAMINFO
 * (42 bytes: 4096-sample blocks, 48 kHz as flac.cpp:311, MD5 unknown);
 * rpp_flac_parse_stream reads any stream's metadata blocks and returns the
 * offset of its first frame (or an RPP_* error).
 */
typedef struct rpp_flac_frame {
  uint64_t uncompressed_bytes;
  uint32_t num_channels;
  uint32_t bits_per_sample;
  uint32_t flags;
} rpp_flac_frame;

typedef struct rpp_flac_stream_info {
  uint32_t min_blocksize, max_blocksize;
  uint32_t sample_rate, channels, bits_per_sample;
  uint64_t total_samples;
} rpp_flac_stream_info;

size_t rpp_flac_frame_header(const rpp_flac_frame* f, uint8_t* out);
long rpp_flac_parse_frame(const uint8_t* in, size_t in_len, rpp_flac_frame* f);
size_t rpp_flac_stream_header(uint32_t channels, uint32_t bps, uint64_t nsamples, uint8_t* out);
long rpp_flac_parse_stream(const uint8_t* in, size_t len, rpp_flac_stream_info* info);

/*
 * FLAC frames on the device (replaces the libFLAC stream encoder /
 * decoder calls of flac.cpp:306-349 and :442-472).
 *
 * rpp_flac_encode: nsamples interleaved frames of `channels` int32 samples
 * of `bps` significant bits (8..32; channels 1..8, flac.cpp:243-245) ->
 * FLAC frames of 4096 samples (fixed and LPC predictors, stereo
 * decorrelation, partitioned Rice codes, CRC-8 / CRC-16) back to back at d_out
 * (rpp_flac_frame_bound bytes per frame at most); *d_total = their size.
 * Workspace: rpp_flac_encode_workspace_bytes.
 *
 * rpp_flac_decode: the frames of a stream (after its metadata blocks) ->
 * nsamples interleaved frames of int32 samples; every RFC 9639 frame kind is
 * accepted.  Frame starts are found by a sync-code scan: at most
 * max_candidates of them are kept; *d_ncand receives how many there were
 * (more than max_candidates: call again with a larger workspace).  *d_status:
 * RPP_OK, RPP_TRUNCATED_INPUT or RPP_INVALID_ARGUMENT (a frame that does not
 * parse or fails its CRC).  Workspace: rpp_flac_decode_workspace_bytes.
 */
uint64_t rpp_flac_frame_bound(uint32_t channels, uint32_t bps);
uint64_t rpp_flac_encode_workspace_bytes(uint64_t nsamples, uint32_t channels, uint32_t bps);
int rpp_flac_encode(const int32_t* d_samples, uint64_t nsamples, uint32_t channels, uint32_t bps, uint8_t* d_out,
                    uint64_t* d_total, void* d_workspace, uint64_t workspace_bytes, void* stream);
/* rpp_flac_encode at a libFLAC compression level (0..8: levels 0-2 fixed
 * predictors only, 3 LPC up to order 6, 4-6 up to 8, 7-8 up to 12; Rice
 * partition orders up to 3 / 4 / 5) and with `exhaustive` (every LPC order
 * coded, the cheapest kept; else libFLAC's expected-bits estimate picks the
 * order) -- FLAC__stream_encoder_set_compression_level / _set_do_exhaustive_
 * model_search as flac.cpp:312-313 calls them.  rpp_flac_encode is level 5. */
int rpp_flac_encode_ex(const int32_t* d_samples, uint64_t nsamples, uint32_t channels, uint32_t bps, uint32_t level,
                       uint32_t exhaustive, uint8_t* d_out, uint64_t* d_total, void* d_workspace,
                       uint64_t workspace_bytes, void* stream);
/* Several blocks in one launch (DwarFS compresses one block per call,
 * flac.cpp:284-349; a batching caller, as the ricepp facade does for ricepp,
 * joins them): block b is h_nsamples[b] interleaved frames of h_channels[b]
 * int32 samples of h_bps[b] bits at d_samples + h_in_off[b] (host arrays: the
 * launch needs the frame count).  Its FLAC frames (numbered from 0) are
 * written to d_out[d_out_off[b], d_out_off[b + 1]) (d_out_off: device,
 * nblocks + 1 entries), byte-identical to rpp_flac_encode_ex of that block
 * alone.  Workspace: rpp_flac_encode_batch_workspace_bytes. */
uint64_t rpp_flac_encode_batch_workspace_bytes(uint32_t nblocks, const uint64_t* h_nsamples, const uint32_t* h_channels,
                                               const uint32_t* h_bps);
int rpp_flac_encode_batch(const int32_t* d_samples, uint32_t nblocks, const uint64_t* h_in_off,
                          const uint64_t* h_nsamples, const uint32_t* h_channels, const uint32_t* h_bps,
                          uint32_t level, uint32_t exhaustive, uint8_t* d_out, uint64_t* d_out_off, void* d_workspace,
                          uint64_t workspace_bytes, void* stream);
uint64_t rpp_flac_decode_workspace_bytes(uint64_t nbytes, uint32_t channels, uint32_t bps, uint32_t max_blocksize,
                                         uint32_t max_candidates);
int rpp_flac_decode(const uint8_t* d_frames, uint64_t nbytes, uint32_t channels, uint32_t bps,
                    uint32_t max_blocksize, uint64_t nsamples, int32_t* d_out, int32_t* d_status,
                    uint32_t max_candidates, void* d_workspace, uint64_t workspace_bytes, uint32_t* d_ncand,
                    void* stream);
/* Several streams' frames decoded in one sequence of launches (the
 * reference decompresses one block per call, flac.cpp:405-489; a batching
 * caller joins them as the ricepp facade does): stream b is h_nbytes[b]
 * bytes of frames at d_frames + h_in_off[b] with its STREAMINFO's channels,
 * bps, max block size and h_nsamples[b] samples per channel, decoded to
 * d_out + h_out_off[b] (int32 elements) with d_status[b] and d_ncand[b] as
 * rpp_flac_decode gives them for that stream alone -- byte for byte the
 * same.  Host arrays (the launches need the sizes); nblocks <= 65535.
 * Workspace: rpp_flac_decode_batch_workspace_bytes. */
uint64_t rpp_flac_decode_batch_workspace_bytes(uint32_t nblocks, const uint64_t* h_nbytes, const uint32_t* h_channels,
                                               const uint32_t* h_bps, const uint32_t* h_max_blocksize,
                                               const uint32_t* h_max_candidates);
int rpp_flac_decode_batch(const uint8_t* d_frames, uint32_t nblocks, const uint64_t* h_in_off,
                          const uint64_t* h_nbytes, const uint32_t* h_channels, const uint32_t* h_bps,
                          const uint32_t* h_max_blocksize, const uint64_t* h_nsamples, int32_t* d_out,
                          const uint64_t* h_out_off, int32_t* d_status, const uint32_t* h_max_candidates,
                          void* d_workspace, uint64_t workspace_bytes, uint32_t* d_ncand, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RICEPP_AMD_H */
