/*
 * brotli_amd -- MI355X (gfx950) Brotli encode/decode engine: the C ABI.
 *
 * This is the drop-in boundary for countertype/brotli-lib's public surface
 * (package.json:7-23 exports `.`, `./encode`, `./decode`):
 *
 *   brotliEncode(input, {quality, lgwin, mode, sizeHint})  src/encode/encode.ts:22-27,50-90  -> mib_encode
 *   new BrotliEncoder(opts).update(chunk) / .finish()      src/encode/encode.ts:290-409      -> mib_encoder_*
 *   brotliDecode(data, {maxOutputSize, customDictionary} | outputSize)
 *                                                          src/decode/decode.ts:13-65        -> mib_decode
 *   brotliDecodedSize(data)                                src/decode/decode.ts:9-11         -> mib_decoded_size
 *   EncoderMode {GENERIC 0, TEXT 1, FONT 2}                src/encode/enc-constants.ts:56-60 -> MIB_MODE_*
 *
 * plus batch entry points (host or device-resident buffers) that shard independent buffers
 * over the GPU.  Every call is synchronous.  The host-buffer entry points
 * share one default context and are serialised internally (safe from several threads); a
 * mib_ctx / mib_encoder handle must not be used by two threads at once.
 * All compute runs on the GPU: there is no CPU fallback, a missing device is an error.
 *
 * Return codes: 0 = success; the reference decoder's own negative codes (-1..-30,
 * engine.ts makeError sites) so a host shim can throw the identical
 * "Brotli error code: N"; MIB_E_* (<= -100) for conditions of this engine.
 */
#ifndef BROTLI_AMD_H_
#define BROTLI_AMD_H_
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define MIB_MODE_GENERIC 0
#define MIB_MODE_TEXT 1
#define MIB_MODE_FONT 2

#define MIB_E_NO_DEVICE (-100)      /* no usable gfx950 device / HIP runtime error */
#define MIB_E_INVALID_ARG (-101)
#define MIB_E_OUT_OF_MEMORY (-102)
#define MIB_E_OUTPUT_LIMIT (-103)   /* decoded size exceeds maxOutputSize (decode.ts:46-62) */
#define MIB_E_NEED_SPACE (-104)     /* device buffer too small (batch/device APIs) */
#define MIB_E_JS_RANGE_ERROR (-105) /* the reference would throw a JS RangeError here */
#define MIB_E_JS_TYPE_ERROR (-106)  /* the reference would throw a JS TypeError here */
#define MIB_E_NO_PROGRESS (-107)    /* decoder iteration guard tripped (never on valid input) */

typedef struct {
  int quality;        /* 0..11, default 11 (clamped like encode.ts:57-62) */
  int lgwin;          /* 10..24, default 22 */
  int mode;           /* MIB_MODE_* */
  uint64_t size_hint; /* accepted, no effect (as in the reference) */
  /* customDictionary (extension: the reference's BrotliEncodeOptions, encode.ts:22-27, has
   * none; this is the encoder side of brotliDecode's customDictionary, decode.ts:13-35).
   * Copies into it are addressed the way the reference decoder resolves a compound
   * dictionary (engine.ts:142-159,903-1011): distance > max distance.  That decoder only
   * accepts a copy that ends exactly at the dictionary's last byte, so the encoder only
   * emits such copies; the stream then decodes with the same dictionary, and only with it.
   * Host memory, borrowed for the call (BrotliEncoder keeps its own copy). NULL: none. */
  const uint8_t *dict;
  uint64_t dict_len;
  /* BrotliEncoder only (extension): 0 = the reference's cadence (encode.ts:366-374: every
   * update() encodes each complete 2^lgblock block it has and returns its bytes); N > 0 =
   * throughput mode: input gathers until at least N bytes (whole blocks) are pending, and the
   * device encode then grows with the stream (up to 256 MiB) -- update() may return nothing
   * for a while and finish() returns the rest. */
  uint64_t stream_chunk;
} mib_enc_opts;

typedef struct { uint8_t *data; size_t size; } mib_buf;          /* library-allocated result */
typedef struct { const uint8_t *data; size_t size; } mib_span;   /* borrowed input */

/* defaults of createDefaultParams (enc-constants.ts:209-233) */
void mib_enc_opts_default(mib_enc_opts *o);

/* Select the device (default 0) and warm the engine up; optional. */
int mib_init(int device);
/* Human-readable message for a return code ("Brotli error code: N" for the reference's codes). */
const char *mib_strerror(int code);

/* brotliEncode (encode.ts:50-90). */
int mib_encode(const uint8_t *in, size_t n, const mib_enc_opts *o, mib_buf *out);

/* brotliDecode (decode.ts:18-65).  exact_out >= 0: the legacy numeric `outputSize`
 * signature (truncate / zero-pad to it); -1: none.  max_out: `maxOutputSize`, -1 = none.
 * dict: `customDictionary` (compound-dictionary semantics, engine.ts:142-159), may be NULL.
 * On MIB_E_OUTPUT_LIMIT no data is returned and out->size holds the size that exceeded
 * the limit (the header's size before decoding, the decoded length after). */
int mib_decode(const uint8_t *in, size_t n, const uint8_t *dict, size_t dict_n, int64_t max_out,
               int64_t exact_out, mib_buf *out);

/* brotliDecodedSize (decode.ts:9-11 -> engine.ts:2155-2192): -1 when unknown. */
int64_t mib_decoded_size(const uint8_t *in, size_t n);

/* BrotliEncoder (encode.ts:290-490): update() returns the newly completed bytes.  The
 * encoder keeps its 2^lgwin window of history in HBM, so matches reach across update()
 * calls; input is encoded in whole 2^lgblock blocks: by default each update() encodes the
 * complete blocks it has (the reference's cadence), with mib_enc_opts.stream_chunk several
 * MiB per device pass (throughput mode). */
typedef struct mib_encoder mib_encoder;
mib_encoder *mib_encoder_new(const mib_enc_opts *o);
int mib_encoder_update(mib_encoder *e, const uint8_t *in, size_t n, mib_buf *out);
int mib_encoder_finish(mib_encoder *e, mib_buf *out);
void mib_encoder_free(mib_encoder *e);
/* k independent encoders (distinct handles) advance by one chunk each in one launch sequence
 * (encoders with equal options share it); out[i] is encoder i's update() result. */
int mib_encoder_update_batch(mib_encoder *const *e, const mib_span *in, size_t k, mib_buf *out);

/* Batches of independent buffers in host memory; one result (and status) per buffer. */
int mib_encode_batch(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status);
int mib_decode_batch(const mib_span *in, size_t k, mib_buf *out, int *status);
/* The same batches sharded over GPUs (SURVEY.md §8(b),(e)): n_gpus shards (<= 0: one per
 * visible device), size-balanced, one host thread and context per shard, shard s on device
 * s % device count; results in input order.  Safe from several threads (calls serialise). */
int mib_encode_batch_n(const mib_span *in, size_t k, const mib_enc_opts *o, int n_gpus, mib_buf *out, int *status);
int mib_decode_batch_n(const mib_span *in, size_t k, int n_gpus, mib_buf *out, int *status);
/* Visible HIP devices (0 without a GPU). */
int mib_device_count(void);
/* Diagnostics: the hardware property the match finder's bucket sort relies on for its
 * stability (the lanes of one wave's returning LDS atomic on one address are served in lane
 * order): lanes that broke it over `trials` random collision patterns (0 expected), < 0 on a
 * HIP error. */
int64_t mib_selftest_lds_atomic_order(int trials);
/* The library runs that self-test once per device and, where it fails, ranks the sort's
 * items by wave ballots instead (same stream bytes, slower).  Test hook: force = 1 makes
 * every device take the ballot ranking, 0 restores the self-test's choice. */
void mib_force_ballot_rank(int force);
/* Diagnostic (tests): non-zero makes mib_encode_batch_n / mib_decode_batch_n shard even when one
 * device is visible (by default a single device runs them as mib_encode_batch / mib_decode_batch,
 * one launch sequence). */
void mib_force_shards(int force);
/* Diagnostic (tests): non-zero turns the q10+ parse's distance-cache candidates off (the
 * parse then prices only last-distance copies, short codes 1-15 arise only where codes_kernel
 * finds a chosen distance in the ring), so a test can show what the candidates change; 0
 * restores them. */
void mib_force_no_dp_cache(int off);

void mib_buf_free(mib_buf *b);
/* The allocator behind every mib_buf the library returns (default malloc / free), in the
 * convention of brotli's own C API (brotli_alloc_func / brotli_free_func with an opaque
 * pointer, c/include/brotli/types.h): a binding can hand results over without a copy (the
 * Python mirror allocates its bytes objects this way).  Process-wide; set it before any
 * other call and free every buffer with the allocator that made it.  NULL, NULL: malloc /
 * free again.  alloc may return NULL (MIB_E_OUT_OF_MEMORY). */
typedef void *(*mib_alloc_func)(void *opaque, size_t size);
typedef void (*mib_free_func)(void *opaque, void *address);
void mib_set_allocator(mib_alloc_func alloc_func, mib_free_func free_func, void *opaque);

/* ---- device-resident batches (inputs already in HBM; used by bench.py and the
 *      multi-GPU driver).  d_* are device pointers on the context's device; offsets are
 *      host arrays of k+1 entries; `stream` is a hipStream_t (NULL = the context's own). */
typedef struct mib_ctx mib_ctx;
mib_ctx *mib_ctx_new(int device);
void mib_ctx_free(mib_ctx *c);
/* Packs the k compressed streams back to back into d_out (capacity out_cap) and fills
 * out_offsets[0..k].  Returns 0, or MIB_E_NEED_SPACE. */
int mib_ctx_encode(mib_ctx *c, const mib_enc_opts *o, const uint8_t *d_in, const uint64_t *in_offsets,
                   size_t k, uint8_t *d_out, uint64_t out_cap, uint64_t *out_offsets, void *stream);
/* Decodes k streams; stream i's output goes to d_out + out_offsets[i] with capacity
 * out_offsets[i+1] - out_offsets[i].  out_sizes[i] / status[i] filled (host arrays). */
int mib_ctx_decode(mib_ctx *c, const uint8_t *d_in, const uint64_t *in_offsets, size_t k, uint8_t *d_out,
                   const uint64_t *out_offsets, int64_t *out_sizes, int *status, void *stream);
/* Per-kernel device time of the last mib_ctx_* call (ms, HIP events on the launch stream). */
typedef struct { char name[32]; double ms; uint32_t launches; } mib_kernel_time;
int mib_ctx_kernel_times(mib_ctx *c, mib_kernel_time *out, int max);
/* on: 0 off, 1 every kernel, 2 the decoder's kernels only (one event pair a decode call; the
 * encoder's ~25 event pairs a call are overhead a small call notices). */
void mib_ctx_set_profiling(mib_ctx *c, int on);
/* The context behind the host-buffer entry points (mib_encode, mib_decode, the batches,
 * BrotliEncoder), created on first use (NULL without a device): for profiling them.  Its
 * kernel times accumulate over those calls until mib_ctx_clear_times. */
mib_ctx *mib_default_ctx(void);
void mib_ctx_clear_times(mib_ctx *c);
/* WOFF2 'glyf' transform (the FONT-mode caller, reference README.md:63;
 * W3C WOFF2 section 5.1): the glyf + loca tables of the TrueType font `ttf` become the
 * transformed glyf table (header, the seven streams, the overlap-simple bitmap), byte for
 * byte what fontTools' WOFF2GlyfTable.transform produces.  MIB_E_INVALID_ARG for a font
 * without glyf / loca / head / maxp or with a malformed glyph. */
int mib_woff2_transform_glyf(const uint8_t *ttf, size_t n, mib_buf *out);
/* WOFF2 'hmtx' transform (W3C WOFF2 section 5.4; fontTools WOFF2HmtxTable.transform): flags,
 * the advance widths and whichever left-side-bearing array does not equal the glyphs' xMin.
 * Returns 0 with out->size = 0 when both arrays differ (no transform: the table is stored
 * as is).  The transformed loca table is empty (WOFF2 section 5.3): nothing to compute. */
int mib_woff2_transform_hmtx(const uint8_t *ttf, size_t n, mib_buf *out);

/* Part-parallel decoding (streams this encoder marked with a part index):
 * how many streams a context (NULL: the default one) decoded part-parallel, and how many of
 * those it sent back to the serial decoder because a part did not check out. Diagnostic. */
void mib_part_stats(mib_ctx *c, uint64_t *parallel, uint64_t *fallback);

#ifdef __cplusplus
}
#endif
#endif
