/*
 * ORACLE -- TEST INFRASTRUCTURE ONLY (see oracle_decode.c / oracle_encode.c headers).
 * CPU restatement of countertype/brotli-lib's encode/decode algorithms, used as the
 * checker for the HIP path and as bench.py's cpu_baseline.  Never linked by the product.
 */
#ifndef BROTLI_ORACLE_H_
#define BROTLI_ORACLE_H_
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* engine.ts:2155 peekDecodedSize: decoded size of a single-ISLAST-metablock stream, else -1/0 */
int64_t oracle_peek_decoded_size(const uint8_t *in, size_t n);

/* engine.ts:2197 brotliDecode.  out_size > 0: decode into an exact buffer of that size
 * (truncate / zero-pad, trailing checks skipped, as the reference).  Returns 0 or the
 * reference's negative error code; *out is malloc'ed (free with oracle_free). */
int oracle_decode(const uint8_t *in, size_t n, const uint8_t *dict, size_t dict_n,
                  int64_t out_size, uint8_t **out, size_t *out_n);
/* decode and record the decoder state (parts.h PartEntry layout, 72 bytes each) at the
 * command boundaries / metablock headers at the ascending output positions pos[0..npos) */
int oracle_decode_probe(const uint8_t *in, size_t n, const uint64_t *pos, size_t npos, void *states);
/* static-dictionary word references decoded so far by this process (test instrumentation) */
uint64_t oracle_word_refs(void);
uint64_t oracle_compound_refs(void);
/* out[4]: the copies decoded on this thread since the last call, by distance code: implicit
 * (command code < 128), explicit code 0, short codes 1-15, explicit distances (>= 16) */
void oracle_dist_code_counts(uint64_t *out);
void oracle_max_block_types(int *out);   /* largest (literal, command, distance) block type counts decoded (clears) */

/* encode.ts:50 brotliEncode (bugs A,B fixed = the survey's "ref-fixed"; C,E fixed too).
 * quality 0..11, lgwin 10..24, mode 0 GENERIC / 1 TEXT / 2 FONT. */
int oracle_encode(const uint8_t *in, size_t n, int quality, int lgwin, int mode,
                  uint8_t **out, size_t *out_n);

/* createHqZopfliBackwardReferences pass 1: every position's findAllMatches list (ref-fixed
 * binary tree, hash-binary-tree.ts:57-227), flat: i, count, (distance, length) x count. */
int64_t oracle_bt_matches(const uint8_t *in, size_t n, int lgwin, uint32_t *out, size_t cap);

void oracle_free(void *p);

#ifdef __cplusplus
}
#endif
#endif
