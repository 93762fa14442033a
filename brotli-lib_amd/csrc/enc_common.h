// brotli_amd encoder: definitions shared by the encoder's kernel files (enc_*.hip) and
// the host orchestration (encode.hip).  See encode.hip for the pipeline overview.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "parts.h"

#ifndef RFC_CONST
#define RFC_CONST static __device__ const
#endif
#include "rfc_tables.h"

namespace mib {
namespace enc {

constexpr uint32_t kSegBits = 16;
constexpr uint32_t kSeg = 1u << kSegBits;     // 64 KiB parse segments
// staircase entries kept per position (the longest ones).  4 by measurement (6 and 8
// change C4 / C3 by < 0.05 % for more record traffic and a slower parse; the reference's own
// q11 parse, restated by the oracle, gains nothing from more than 4 either); MIB_MAX_MATCHES=6|8
// builds the wider records for that A/B.
#ifndef MIB_MAX_MATCHES
#define MIB_MAX_MATCHES 4
#endif
constexpr int kMaxMatches = MIB_MAX_MATCHES;
static_assert(kMaxMatches == 4 || kMaxMatches == 6 || kMaxMatches == 8, "records of 4, 6 or 8 entries");
constexpr int kMatchRec = kMaxMatches;        // u32 per position record: the matches, 0 = none (16 B at 4)
constexpr uint32_t kMatchLenSat = 255;        // a match is (length:8 | distance:24); 255 = "255 or more"
constexpr int kLongCopy = 200;                // copies longer than this are taken outright (the
                                              // reference's MAX_ZOPFLI_LEN is 325 at q11, 150 at q10,
                                              // enc-constants.ts:32-33)
constexpr uint32_t kMaxMetablock = 1u << 24;  // encode.ts:206
constexpr uint32_t kHashBits = 17;            // bucket hash bits (hashBytes4, match.ts:162-172)
constexpr int kHashBytes = 6;                  // bytes a bucket key covers (see hashn)
constexpr uint32_t kInvalidKey = 1u << kHashBits;   // the sort key of positions without kHashBytes bytes
// Streaming history (BrotliEncoder across update() calls): per encoder, for every hash bucket
// the stream positions of its kHistWays most recent earlier occurrences, newest first
// (the reference keeps a hash chain over its ring, hash-chains.ts / encode.ts:354-374).
constexpr int kHistWays = 16;
constexpr uint32_t kNoPos = 0xFFFFFFFFu;              // (a history slot with no position)
constexpr int kHdrBytes = 2048;               // metablock header: block-switch codes, context maps (not the trees)
constexpr int kTreeBytes = 1024;              // one serialised prefix code
constexpr int kLitCtx = 64;                   // literal contexts (RFC 7932 section 7.1)
constexpr int kDistCtx = 4;                   // distance contexts (copy length 2, 3, 4, >4)
// Block splitting (block-splitter.ts): up to kMaxBT block types per category, decided per
// metablock over 8 KiB units of commands (kSubBits), kSubPerSeg units per parse segment.
constexpr int kMaxBT = 8;
constexpr uint32_t kSubBits = 13;
constexpr int kSubPerSeg = 1 << (kSegBits - kSubBits);
constexpr int kSplitWideUnits = 256;          // literal metablocks of up to 2 MiB (units) may take 8
                                              // types, longer ones 4 (enc_entropy.hip split_k)
constexpr int kSubHist = 256 + 704 + 128;      // a unit's literal | command | distance-code histograms
constexpr int kMaxLitTrees = 64;              // literal prefix codes per metablock (decoder tables stay in LDS)
// code slots: literal (type, cluster) | command (type) | distance (type, cluster)
constexpr int kLitSlots = kMaxBT * kLitCtx;
constexpr int kCmdSlot = kLitSlots;
constexpr int kDistSlot = kCmdSlot + kMaxBT;
constexpr int kTreeSlots = kDistSlot + kMaxBT * kDistCtx;
constexpr int kBlock = 256;                   // threads of the per-segment entropy / emit blocks
constexpr int kMaxPieceShift = 7;             // parse pieces per segment: at most 2^7 (encode.hip)
// a segment's commands fill at most kSeg / 2 + 4 + (2 << kMaxPieceShift) slots (its cmds span,
// encode.hip); sizes_kernel records their bits per tile of kEmitTile commands, so emit_kernel
// can write a segment's tiles from blocks of their own
constexpr int kEmitTile = 512;
constexpr int kEmitTiles = (int)((kSeg / 2 + 4 + (2u << kMaxPieceShift) + kEmitTile - 1) / kEmitTile);

struct Job {                // one stream (or streaming chunk) to encode
  const uint8_t *data;      // its bytes (device)
  uint32_t n;
  uint32_t pos_base;        // global position index of byte 0 (sort / per-position arrays)
  uint32_t seg_base;        // first segment
  uint32_t nseg;
  uint32_t mb_base;         // first metablock
  uint32_t nmb;
  uint32_t lgwin;
  uint32_t npostfix, ndirect;
  uint32_t uncompressed;    // 1: quality 0 / n < 64 path; 2: compressed form was larger
  uint32_t hdr_lgwin;       // window bits written before the first metablock, 0 = none
  uint32_t final_;          // last chunk of the stream: ISLAST metablock (else a byte-aligning flush)
  int32_t dc_in[4];         // the decoder's distance ring at the start (streaming continues it)
  uint32_t prev_bytes;      // the two bytes before data[0] (streaming: the previous chunk's tail), p1 | p2 << 8
  int32_t dc_out[4];        // and after the last command
  uint32_t hist;            // streaming: bytes of the stream before data[0] that copies may reach
  uint32_t abs_base;        // streaming: stream position of data[0] (mod 2^32)
  uint32_t win_abs;         // min(stream position of data[0], 2^24): the window a dictionary
                            // distance lies beyond is min(win_abs + p, max backward), exact
                            // past 4 GiB of stream too (max backward < 2^24)
  uint32_t *hist_tab;       // streaming: the encoder's bucket table of earlier positions, or null
  uint32_t dict;            // 1: static-dictionary references allowed (one-shot, lgwin <= 22, q >= 10)
  uint32_t dict_span;       // ... at stream positions below this (where the window is still short)
  uint32_t parts;           // 1: part index (parts.h) -- external copy sources lag, index block first
  uint32_t idx_payload;     // part index: metadata payload bytes
  uint32_t part_bits;       // part index: log2 of the part size (>= kSegBits)
  uint32_t part_lag;        // part index: how far an external copy source lags (bytes)
  uint64_t idx_bits;        // part index: bits before the first metablock (window bits + index block)
  uint64_t out_base;        // streaming: stream bytes emitted before this chunk
  uint64_t out_off;         // byte offset of its scratch output slice
  uint64_t out_cap;
  uint64_t total_bits;      // written by offsets / stored
  const uint8_t *cdict;     // custom dictionary (device), or null (see kCDictMark)
  uint32_t cdict_len;
  uint32_t cdict_tail4;     // its last four bytes (little endian)
  uint32_t font;            // FONT mode (last-distance copies pass, 4-byte keys)
  uint32_t hq;              // quality >= 10 (context mode rule)
  uint32_t binary;          // set by context_mode_kernel: some metablock's literals are not UTF-8
                            // text (the parse's distance-cache candidates run there)
};

// Per 64 KiB of global positions: where its stream's bytes are, so the match finder's gather
// needs one lookup, not the segment's stream and then its Job (a dependent pair of loads)
struct SegRef {
  const uint8_t *base;      // the stream's data - pos_base (byte of global position g: base + g)
  uint32_t pos_base;        // the stream's first global position
  uint32_t end;             // pos_base + its length (0 bytes for an uncompressed stream)
};

// Custom-dictionary copies (mib_enc_opts.dict; the reference decoder's compound dictionary,
// engine.ts:142-159,903-1011).  A copy of length L at stream position p with distance
// d = min(p, max backward distance) + L is read by the decoder from dictionary offset
// dict_len - L: the dictionary's last L bytes (the reference decoder rejects any other
// compound copy, engine.ts:992, so these are the only ones ever emitted).  A match record
// names one by the distance kCDictMark (no window distance is that large) and its exact
// length; the parse turns it into d.  Downstream it is an ordinary copy: it pushes on the
// distance ring and may be repeated by a short code, as in the decoder.
constexpr uint32_t kCDictMark = 0xFFFFFFu;

// Static-dictionary references (RFC 7932 section 8, identity transform):
// a copy whose distance exceeds the decoder's maximum backward distance names the word of
// its length with index distance - (max distance + 1).  Encoder-side such a copy carries
// kDictFlag in its distance (window distances stay below 2^22: dictionary words are only
// used at lgwin <= 22): it never pushes on the distance ring and is always coded with an
// explicit distance code; as a "previous distance" it equals no window distance, so the
// copy after it never takes code 0 by mistake.
constexpr uint32_t kDictFlag = 1u << 23;
constexpr int kDictHashBits = 15;           // word table: buckets by the first 4 bytes
constexpr int kDictWays = 8;                // words per bucket, longest first (length << 16 | index)
__device__ __forceinline__ bool is_dict(uint32_t d) { return (d & kDictFlag) != 0; }
__device__ __forceinline__ uint32_t dict_hash(uint32_t w4) { return (w4 * 0x1E35A7BDu) >> (32 - kDictHashBits); }

// (only streams with dict set carry word references; at lgwin > 22 bit 23 is a distance bit)
__device__ __forceinline__ bool is_word(const Job &jb, uint32_t d) { return jb.dict && is_dict(d); }

struct Seg {
  uint32_t job, start, end;   // stream-local [start, end)
  uint32_t mb;                // metablock (global index)
  uint32_t cmd_off;           // command slice (capacity (end-start)/2 + 20: its parse pieces' slices fit)
  uint32_t ncmd;              // backtrack: copy commands
  uint32_t tail_lits;         // backtrack: literals after the last copy (all of them if none)
  uint32_t last_dist;         // backtrack: distance of the last copy (0: none)
  uint32_t carry_in;          // carry: literals owed by earlier segments of the metablock
  uint32_t prev_dist;         // carry: the decoder's last distance when the segment starts
  uint32_t extra_ins;         // carry: trailing insert-only command of the metablock (0: none)
  uint32_t pieces;            // its parse pieces: first piece index << 3 | log2 of their count
  uint32_t ring_in[4];        // ring_scan: the decoder's distance ring at the segment start, most recent first
  uint64_t bit_off;           // offsets: stream-relative bit position
  uint64_t bits;              // sizes
};

struct Mb {                   // one metablock: block types per category, literal and
                              // distance context modelling (storeMetaBlock, metablock.ts:504-761)
  uint32_t job, start, end;   // stream-local
  uint32_t first_seg, nseg;
  uint32_t is_last;
  uint32_t hdr_bits;          // header bits before the prefix codes (incl. context maps)
  uint32_t ctx_mode;          // literal context mode (chooseContextMode, context.ts:180-227)
  uint32_t nbt[3];            // block types: literal, command, distance
  float split_gain[3];        // the four-type split's saving, a share of the one-type cost (0: no split)
  uint32_t first_count[3];    // symbols in the first block of each category
  uint32_t nlit_t[kMaxBT], ndist_t[kMaxBT];   // prefix codes (clusters) per literal / distance block type
  uint16_t lit_cmap[kLitSlots];            // (type, context) -> literal code slot (type * 64 + cluster)
  uint8_t dist_cmap[kMaxBT * kDistCtx];    // (type, context) -> distance code slot (type * 4 + cluster)
  uint32_t tree_bits[kTreeSlots];
  uint64_t bit_off;           // of the header, stream-relative
};

struct Unit {                 // one block-split unit: the commands of 8 KiB of a segment
  uint32_t nsym[3];           // symbols: literals, commands, distance codes
  uint32_t first[3];          // literals: stream position of its first literal; commands /
                              // distance codes: segment-relative index of its first command
                              // (any / with a distance code) (~0u: none)
  uint32_t sw_count[3];       // block switch before that symbol: the new block's count (0: none)
  uint8_t type[3];            // block type per category
  uint8_t sw_code[3];         // the switch's block type code (RFC 7932 section 6)
  uint16_t pad;
};

struct Cmd {                  // one command with its prefix codes (command.ts:29-208)
  uint32_t ins, copy;         // copy == 0: trailing insert-only command
  uint32_t dist;              // its distance (for the distance ring)
  uint32_t dist_extra;
  uint16_t cmd_prefix, dist_prefix;   // dist_prefix: code | nbits << 10, code 0 = last distance
};

struct RawCmd { uint32_t ins, len, dist; };

// The parse's second-iteration prices (ZopfliCostModel.setFromCommands,
// zopfli-cost-model.ts:68-159): bits per literal, command code and distance code from the
// first parse's commands, one model per stream
struct CostModel {
  float lit[256];
  float cmd[704];
  float dist[128];
};

struct Codes {   // per metablock Huffman codes by slot, and the block-switch codes
  uint8_t ld[kLitSlots][256];
  uint16_t lc[kLitSlots][256];
  uint8_t cd[kMaxBT][704];
  uint16_t cc[kMaxBT][704];
  uint8_t dd[kMaxBT * kDistCtx][128];
  uint16_t dcd[kMaxBT * kDistCtx][128];
  uint8_t btd[3][kMaxBT + 2];   // block type codes
  uint16_t btc[3][kMaxBT + 2];
  uint8_t bcd[3][26];           // block count codes
  uint16_t bcc[3][26];
};

// block count prefix codes (RFC 7932 section 6; engine.ts kBlockLengthOffset / NBits)
static __device__ __constant__ uint32_t kBlkOff[26] = {1,   5,   9,   13,  17,  25,   33,   41,   49,   65,   81,    97,    113,
                                                       145, 177, 209, 241, 305, 369, 497, 753, 1265, 2289, 4337, 8433, 16625};
static __device__ __constant__ uint32_t kBlkBits[26] = {2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 7, 8, 9, 10, 11, 12, 13, 24};
__device__ __forceinline__ int block_count_code(uint32_t count) {
  int c = 0;
  while (c < 25 && kBlkOff[c + 1] <= count) c++;
  return c;
}

// ---------------------------------------------------------------- coding helpers (command.ts)
__device__ __forceinline__ int log2floor_u(uint32_t v) { return 31 - __clz(v); }
// (each kernel file gets its own copy: device code is not linked across files)
static __device__ __constant__ uint32_t kInsBase[24] = {0,   1,   2,   3,   4,   5,    6,    8,    10,   14,   18,   26,
                                                        34,  50,  66,  98,  130, 194,  322,  578,  1090, 2114, 6210, 22594};
static __device__ __constant__ uint32_t kInsExtra[24] = {0, 0, 0, 0, 0, 0, 1, 1,  2,  2,  3,  3,
                                                         4, 4, 5, 5, 6, 7, 8, 9, 10, 12, 14, 24};
static __device__ __constant__ uint32_t kCopyBase[24] = {2,  3,  4,  5,  6,   7,   8,   9,   10,  12,   14,   18,
                                                         22, 30, 38, 54, 70, 102, 134, 198, 326, 582, 1094, 2118};
static __device__ __constant__ uint32_t kCopyExtra[24] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1,  2,  2,
                                                          3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 24};

__device__ __forceinline__ int ins_code(uint32_t n) {
  if (n < 6) return (int)n;
  if (n < 130) {
    int nb = log2floor_u(n - 2) - 1;
    return (nb << 1) + (int)((n - 2) >> nb) + 2;
  }
  if (n < 2114) return log2floor_u(n - 66) + 10;
  if (n < 6210) return 21;
  if (n < 22594) return 22;
  return 23;
}
__device__ __forceinline__ int copy_code(uint32_t n) {
  if (n < 10) return (int)n - 2;
  if (n < 134) {
    int nb = log2floor_u(n - 6) - 1;
    return (nb << 1) + (int)((n - 6) >> nb) + 4;
  }
  if (n < 2118) return log2floor_u(n - 70) + 12;
  return 23;
}
__device__ __forceinline__ int combine_codes(int ic, int cc, bool use_last) {
  int bits64 = (cc & 7) | ((ic & 7) << 3);
  if (use_last && ic < 8 && cc < 16) return cc < 8 ? bits64 : (bits64 | 64);
  int off = 2 * ((cc >> 3) + 3 * (ic >> 3));
  off = (off << 5) + 0x40 + ((0x520D40 >> off) & 0xC0);
  return off | bits64;
}
// prefixEncodeCopyDistance (command.ts:111-135): code | nbits << 10, extra
__device__ __forceinline__ uint32_t dist_prefix(uint32_t dcode, int ndirect, int npostfix, uint32_t *extra) {
  if (dcode < (uint32_t)(16 + ndirect)) {
    *extra = 0;
    return dcode;
  }
  uint32_t dist = (1u << (npostfix + 2)) + (dcode - 16 - (uint32_t)ndirect);
  int bucket = log2floor_u(dist) - 1;
  uint32_t pmask = (1u << npostfix) - 1, postfix = dist & pmask, prefix = (dist >> bucket) & 1;
  uint32_t offset = (2 + prefix) << bucket;
  uint32_t nbits = (uint32_t)(bucket - npostfix);
  *extra = (dist - offset) >> npostfix;
  return (nbits << 10) | (16 + (uint32_t)ndirect + ((2 * (nbits - 1) + prefix) << npostfix) + postfix);
}

// The distance code of a copy at distance d given the decoder's ring r (most recent first)
// when d is not the last distance: a short code 1-15 when d is in the ring or within 3 of its
// first two entries (RFC 7932 section 4; engine.ts DISTANCE_SHORT_CODE_*), else d + 15.
__device__ __forceinline__ uint32_t short_code(uint32_t d, const uint32_t *r) {
  if (d == r[1]) return 1;
  if (d == r[2]) return 2;
  if (d == r[3]) return 3;
  const int64_t a = (int64_t)d - (int64_t)r[0], b = (int64_t)d - (int64_t)r[1];
  if (a >= -3 && a <= 3 && a != 0) return a < 0 ? (uint32_t)(4 + 2 * (-a - 1)) : (uint32_t)(5 + 2 * (a - 1));
  if (b >= -3 && b <= 3 && b != 0) return b < 0 ? (uint32_t)(10 + 2 * (-b - 1)) : (uint32_t)(11 + 2 * (b - 1));
  return d + 15;
}

// a position's record as kMaxMatches words (16-byte or 8-byte vector accesses)
__device__ __forceinline__ void rec_load(const uint32_t *p, uint32_t (&v)[kMaxMatches]) {
  if constexpr (kMaxMatches % 4 == 0) {
#pragma unroll
    for (int q = 0; q < kMaxMatches / 4; q++) {
      const uint4 a = reinterpret_cast<const uint4 *>(p)[q];
      v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kMaxMatches / 2; q++) {
      const uint2 a = reinterpret_cast<const uint2 *>(p)[q];
      v[2 * q] = a.x; v[2 * q + 1] = a.y;
    }
  }
}
__device__ __forceinline__ void rec_store(uint32_t *p, const uint32_t (&v)[kMaxMatches]) {
  if constexpr (kMaxMatches % 4 == 0) {
#pragma unroll
    for (int q = 0; q < kMaxMatches / 4; q++)
      reinterpret_cast<uint4 *>(p)[q] = make_uint4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
  } else {
#pragma unroll
    for (int q = 0; q < kMaxMatches / 2; q++) reinterpret_cast<uint2 *>(p)[q] = make_uint2(v[2 * q], v[2 * q + 1]);
  }
}

__device__ __forceinline__ uint32_t pack_match(uint32_t dist, uint32_t len) {
  return (min(len, kMatchLenSat) << 24) | dist;   // distances are below 2^24 (lgwin <= 24)
}
__device__ __forceinline__ uint32_t match_dist(uint32_t m) { return m & 0xFFFFFFu; }
__device__ __forceinline__ uint32_t match_length(uint32_t m) { return m >> 24; }

// Part index (parts.h): a copy whose source lies in an earlier part (2^bits aligned) must
// end `lag` bytes before the destination's offset in its own part, so the wave decoding that
// earlier part has (in lockstep) already written it.  The longest allowed length of a copy
// at stream position A from distance d (~0u: no limit).
__device__ __forceinline__ uint32_t part_cap(uint32_t A, uint32_t d, uint32_t bits, uint32_t lag) {
  const uint32_t q = A - d;
  if ((q >> bits) == (A >> bits)) return ~0u;
  const uint32_t m = (1u << bits) - 1u, x = A & m, ql = q & m;
  return x >= ql + lag ? x - lag - ql : 0u;
}

__device__ __forceinline__ uint32_t load_u32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
// Bucket key over the first n bytes at p (n = kHashBytes, 4 in FONT mode: encode.hip
// hash_bytes; MIB_HASH_BYTES overrides, 4..6).  The candidate walk is depth-limited (64 at
// q11), so a longer key makes every candidate a match of >= n bytes and lets the walk reach
// farther back: C4 0.3770 -> 0.3706 and find_matches 75 -> 59 ms for 6 bytes (4: the
// reference's hashBytes4, match.ts:162-172); matches of 4-5 bytes are given up, which costs
// glyph data 1.8 %.
__device__ __forceinline__ uint32_t hashn(const uint8_t *p, int n) {
  uint64_t v = load_u32(p);
  for (int i = 4; i < n; i++) v |= (uint64_t)p[i] << (8 * i);
  v <<= 64 - 8 * n;
  return (uint32_t)((v * 0x1E35A7BD1E35A7BDull) >> (64 - kHashBits));
}

// length of the common prefix of a[] and b[], up to limit
__device__ __forceinline__ uint32_t match_len(const uint8_t *a, const uint8_t *b, uint32_t limit) {
  uint32_t m = 0;
  while (m + 4 <= limit) {
    uint32_t x = load_u32(a + m) ^ load_u32(b + m);
    if (x) return m + (__ffs(x) - 1) / 8;
    m += 4;
  }
  while (m < limit && a[m] == b[m]) m++;
  return m;
}

// A block that is a single wave: LDS traffic of a wave is processed in order, so a compiler
// fence at wavefront scope is all the lanes need between dependent LDS steps (a
// workgroup barrier would also drain the outstanding global stores/loads every time).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Serial LSB-first bit writer into a zeroed byte buffer (headers, prefix codes).  Bits gather
// in a register and reach the buffer 32 at a time (OR'ed bytewise: the start need not be byte
// aligned); the rest at flush() or when the writer goes out of scope -- read the buffer after
// either.  (Byte read-modify-writes per put were most of a single metablock's header and tree
// time, r05o.)
struct BitW {
  uint8_t *buf;
  uint64_t pos;        // bits written, the pending ones included
  uint64_t acc = 0;    // pending bits; the first lands at bit pos - nacc
  int nacc = 0;
  __device__ void emit(uint64_t p0, uint32_t v, int n) {   // OR n <= 32 bits of v in at bit p0
    uint8_t *b = buf + (p0 >> 3);
    const int sh = (int)(p0 & 7);
    const uint64_t x = (uint64_t)v << sh;
    const int nb = (sh + n + 7) >> 3;
    for (int i = 0; i < nb; i++) b[i] |= (uint8_t)(x >> (8 * i));
  }
  __device__ void put(int nbits, uint64_t v) {
    while (nbits > 0) {
      const int k = nbits < 32 ? nbits : 32;
      acc |= (v & ((1ull << k) - 1)) << nacc;
      nacc += k;
      pos += k;
      v >>= k;
      nbits -= k;
      if (nacc >= 32) {
        emit(pos - nacc, (uint32_t)acc, 32);
        acc >>= 32;
        nacc -= 32;
      }
    }
  }
  __device__ void flush() {
    if (nacc) emit(pos - nacc, (uint32_t)acc, nacc);
    acc = 0;
    nacc = 0;
  }
  __device__ ~BitW() { flush(); }
};

// encodeWindowBits (bit-writer.ts:172-194)
__device__ __forceinline__ void put_window_bits(BitW &w, int lg) {
  if (lg == 16) w.put(1, 0);
  else if (lg == 17) w.put(7, 1);
  else if (lg > 17) w.put(4, (uint32_t)(((lg - 17) << 1) | 1));
  else w.put(7, (uint32_t)(((lg - 8) << 4) | 1));
}

// the two bytes before stream position p (p1 | p2 << 8): the decoder's ring holds them
__device__ __forceinline__ uint32_t prev2(const Job &jb, uint32_t p) {
  const uint32_t b1 = p >= 1 ? jb.data[p - 1] : (jb.prev_bytes & 0xFF);
  const uint32_t b2 = p >= 2 ? jb.data[p - 2] : (p == 1 ? (jb.prev_bytes & 0xFF) : (jb.prev_bytes >> 8) & 0xFF);
  return b1 | (b2 << 8);
}
// distance context of a copy (RFC 7932 section 7.2; metablock.ts:621)
__device__ __forceinline__ int dist_ctx(uint32_t copy_len) { return copy_len > 4 ? 3 : (int)copy_len - 2; }

// the unit of command q (segment-relative position p of its insert): 8 KiB slices of the segment
__device__ __forceinline__ uint32_t unit_of(const Seg &sg, uint32_t p) {
  const uint32_t c = p < sg.start ? sg.start : (p >= sg.end ? sg.end - 1 : p);
  return (c - sg.start) >> kSubBits;
}
// a block switch: block type code, block count code and its extra bits (storeBlockSwitch,
// metablock.ts:204-220)
__device__ __forceinline__ uint32_t switch_bits(const Codes &cd, int cat, const Unit &u) {
  const int bc = block_count_code(u.sw_count[cat]);
  return cd.btd[cat][u.sw_code[cat]] + cd.bcd[cat][bc] + kBlkBits[bc];
}
// command / distance block switches sit at a command; literal ones at a literal, so a literal
// block can end inside a long insert (glyph data: a few copies, long literal runs)
__device__ __forceinline__ bool switch_at(const Unit &u, int cat, uint32_t q) { return u.sw_count[cat] && q == u.first[cat]; }
__device__ __forceinline__ bool lit_switch_at(const Unit &u, uint32_t lp) { return u.sw_count[0] && lp == u.first[0]; }

// ---------------------------------------------------------------- command items
// A command is coded as a sequence of ITEMS (storeCommandExtra / storeSymbolWithContext /
// BlockEncoder, metablock.ts:273-287,392-501,720-745):
//   item 0            command block switch, command prefix code, insert / copy extra bits,
//                     literal block switch
//   items 1 .. ins    one literal each, under its context (p1, p2 are the input bytes before it)
//   item ins + 1      distance block switch, distance prefix code and extra bits (0 bits for
//                     insert-only and implicit-last-distance commands)
// Items are independent given the command, so literal-heavy segments (glyph data, long
// inserts) spread over the lanes of a block instead of serialising on one lane per command.
// `u` is the block-split unit of the command (by its insert position), q its index.
__device__ __forceinline__ uint32_t item_count(const Cmd &c) { return c.ins + 2; }

__device__ __forceinline__ uint32_t header_bits(const Codes &cd, const Cmd &c, const Unit &u, uint32_t q) {
  const int ic = ins_code(c.ins);
  const int cc = copy_code(c.copy ? c.copy : 2);
  uint32_t bits = cd.cd[u.type[1]][c.cmd_prefix] + kInsExtra[ic] + kCopyExtra[cc];
  if (switch_at(u, 1, q)) bits += switch_bits(cd, 1, u);
  return bits;
}
// (lut, cmap: the context-mode table and the metablock's literal context map, LDS copies in
// the sizes / emit kernels)
__device__ __forceinline__ int literal_tree(const uint16_t *cmap, const uint8_t *lut, const Unit &u, uint32_t p12) {
  return cmap[u.type[0] * kLitCtx + (lut[p12 & 0xFF] | lut[256 + (p12 >> 8)])];
}
__device__ __forceinline__ uint32_t dist_bits(const Codes &cd, const Mb &mb, const Cmd &c, const Unit &u, uint32_t q) {
  if (!c.copy || c.cmd_prefix < 128) return 0;
  uint32_t bits = cd.dd[mb.dist_cmap[u.type[2] * kDistCtx + dist_ctx(c.copy)]][c.dist_prefix & 0x3FF] + (c.dist_prefix >> 10);
  if (switch_at(u, 2, q)) bits += switch_bits(cd, 2, u);
  return bits;
}
// bits of item k of command c (insert at stream position p); su: the segment's units (the
// command's header and distance go by the unit of p, each literal by its own position's)
__device__ __forceinline__ uint32_t item_bits(const Codes &cd, const Mb &mb, const uint16_t *cmap, const uint8_t *lut, const Job &jb,
                                              const Cmd &c, uint32_t p, const Seg &sg, const Unit *su, uint32_t q,
                                              uint32_t k) {
  if (k == 0) return header_bits(cd, c, su[unit_of(sg, p)], q);
  if (k > c.ins) return dist_bits(cd, mb, c, su[unit_of(sg, p)], q);
  const uint32_t lp = p + k - 1;
  const Unit &ul = su[unit_of(sg, lp)];
  return (lit_switch_at(ul, lp) ? switch_bits(cd, 0, ul) : 0u) + cd.ld[literal_tree(cmap, lut, ul, prev2(jb, lp))][jb.data[lp]];
}

// Load-balanced expansion of a batch of at most B commands into their items: off[j] is the
// first item of command j (exclusive scan of the counts), off[nb] the batch's total.
template <int B>
struct ItemMap {
  uint32_t off[B + 1];
  // the command owning item i (i < off[nb]): off[j] <= i < off[j + 1]
  __device__ __forceinline__ uint32_t find(uint32_t i, uint32_t nb) const {
    uint32_t lo = 0, hi = nb;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (off[mid] <= i) lo = mid;
      else hi = mid;
    }
    return lo;
  }
};

// ---------------------------------------------------------------- kernel launchers (host)
void launch_dict_matches(hipStream_t st, const Job *jobs, int njobs, uint32_t span, const uint32_t *dict_tab,
                         const uint8_t *dict_data, uint32_t *matches);
void launch_cdict_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, uint32_t total, uint32_t *matches);
void launch_find_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref,
                         const uint32_t *skeys, const uint32_t *svals, uint32_t total, int depth, uint32_t max_dist,
                         bool hist, bool parts, uint32_t *matches);
void launch_near_matches(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref, uint32_t total,
                         uint32_t max_dist, bool hist, bool parts, uint32_t *matches);
void launch_lit_histo(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, uint32_t *lit_h);
void launch_hist_update(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const uint32_t *skeys,
                        const uint32_t *svals, uint32_t total);
size_t cost_model_hist_bytes(int njobs);
void launch_cost_model(hipStream_t st, const Job *jobs, int njobs, const Seg *segs, int nsegs, const RawCmd *raw,
                       uint32_t *hist, CostModel *model);
void launch_dp(hipStream_t st, const Job *jobs, const Seg *segs, int nsegs, const uint32_t *lit_h, const CostModel *model,
               const uint32_t *matches, uint64_t *choice, bool cdict, bool font, const uint32_t *words, uint32_t *ring_hist,
               const Mb *mbs);
size_t dp_ring_hist_bytes(int nsegs);
void launch_any_binary(hipStream_t st, const Job *jobs, int njobs, uint32_t *flag);
void launch_words(hipStream_t st, const Job *jobs, const uint32_t *pos_job, const SegRef *seg_ref, uint32_t total, uint32_t *words);
void launch_backtrack(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const uint64_t *choice, RawCmd *raw);
void launch_carry(hipStream_t st, Job *jobs, int njobs, Seg *segs, const Mb *mbs);
void launch_derive_segs(hipStream_t st, const Seg *segs, int nsegs, uint32_t sample, Seg *d_sample, Seg *pieces);
void launch_merge_pieces(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const Seg *pieces, RawCmd *raw);
void launch_rep(hipStream_t st, const Job *jobs, Seg *segs, int nsegs, const CostModel *model, RawCmd *raw, uint32_t *cnts);
size_t sort_ws_bytes(uint32_t total);
void launch_sort(hipStream_t st, const Job *jobs, const uint32_t *pos_job, int njobs, uint32_t total, int hb, void *ws,
                 uint32_t *tmp_k, uint32_t *tmp_v, uint32_t *skeys, uint32_t *svals);
void launch_codes(hipStream_t st, const Job *jobs, const Seg *segs, const Mb *mbs, int nsegs, const RawCmd *raw, Cmd *cmds,
                  uint32_t *cmd_pos, Unit *units, uint32_t *unit_h);
// (side: a second stream the caller forks to and joins from; the launcher puts the launch
// that is independent of the one on st there -- st itself when there is none)
void launch_split(hipStream_t st, hipStream_t side, const Job *jobs, Mb *mbs, int nmbs, Unit *units,
                  const uint32_t *unit_h, Codes *codes, int max_units, int max_short_units);
void launch_histo(hipStream_t st, const Job *jobs, const Seg *segs, const Mb *mbs, int nsegs, const Cmd *cmds,
                  const uint32_t *cmd_pos, const Unit *units, uint32_t *hl, uint32_t *hc, uint32_t *hd);
void launch_dist_ring(hipStream_t st, Job *jobs, int njobs, const Seg *segs, const Cmd *cmds);
void launch_context_mode(hipStream_t st, const Job *jobs, Mb *mbs, int nmbs);
void launch_cluster(hipStream_t st, const Job *jobs, Mb *mbs, int nmbs, uint32_t *hl, uint32_t *hd);
void launch_huffman(hipStream_t st, hipStream_t side, const Job *jobs, Mb *mbs, int nmbs, const uint32_t *hl,
                    const uint32_t *hc, const uint32_t *hd, Codes *codes, uint8_t *trees, uint8_t *hdr);
void launch_sizes(hipStream_t st, const Job *jobs, Seg *segs, const Mb *mbs, int nsegs, const Cmd *cmds,
                  const uint32_t *cmd_pos, const Codes *codes, const Unit *units, uint32_t *tile_bits);
void launch_offsets(hipStream_t st, Job *jobs, int njobs, Mb *mbs, Seg *segs, uint8_t *out);
void launch_emit(hipStream_t st, const Job *jobs, const Mb *mbs, int nmbs, const Seg *segs, int nsegs, const Cmd *cmds,
                 const uint32_t *cmd_pos, const Codes *codes, const Unit *units, const uint32_t *tile_bits,
                 const uint8_t *trees, const uint8_t *hdr, uint8_t *out);
void launch_stored(hipStream_t st, Job *jobs, int njobs, uint8_t *out);
struct PushSum;
void launch_ring_scan(hipStream_t st, Job *jobs, int njobs, Seg *segs, int nsegs, const RawCmd *raw, PushSum *push);
void launch_part_index(hipStream_t st, const Job *jobs, int njobs, const Mb *mbs, const Seg *segs, int nsegs,
                       const Cmd *cmds, const Unit *units, PushSum *push, uint8_t *out);
size_t part_push_bytes();
void launch_pack(hipStream_t st, const Job *jobs, int njobs, uint64_t out_pos, uint64_t out_cap, uint64_t *dst_off,
                 const uint8_t *src, uint8_t *dst);

}  // namespace enc
}  // namespace mib
