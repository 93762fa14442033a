// brotli_amd: RFC 7932 stream decoder for gfx950, one wave (64 lanes) per stream.
//
// Semantics are those of the reference decoder (countertype/brotli-lib
// src/decode/engine.ts, a port of Google's Java decoder) so that output bytes AND error
// codes are identical, including on corrupted input:
//   * the 4,160-byte input window refilled when halfOffset > 2030 (engine.ts:1764-1790),
//     kept here in LDS and refilled cooperatively by the wave; its stale bytes after the
//     end of input decide which error a truncated stream raises;
//   * the ring buffer sized by maybeReallocateRingBuffer (:608-630), flushed at the fence
//     (:1477-1497) into the output, kept in a per-block HBM scratch slice;
//   * the command / literal / distance / copy state machine of decompress (:1012-1517),
//     including its literal batching (:1166, :1221) -- with Bug J fixed (a zero
//     batch after end of input spins forever in the reference);
//   * brotliDecode's output modes (:2197-2257): a known size (one pass, truncate/zero-pad,
//     trailing checks skipped) or chunks of 16 KiB doubling to 4 MiB.
//
// GPU mapping: the bit-serial part (Huffman symbol reads) runs wave-uniform -- every lane
// computes the same state, reads broadcast from LDS/L1 -- and the byte-parallel parts
// (window refill, Huffman table replication, LZ77 copies, uncompressed copies, ring
// flushes) are spread over the 64 lanes.  Parallelism across streams comes from the grid:
// a persistent grid of one-wave workgroups walks the job list.
#include <hip/hip_runtime.h>

#include "common.h"
#include "parts.h"
#define RFC_CONST static __device__ const
#include "rfc_tables.h"

namespace mib {

__device__ const uint8_t kDictionary[RFC_DICT_SIZE] = {
#include "rfc_dictionary.inc"
};

__constant__ int16_t kCmdLut[704 * 4];   // engine.ts:65-90, filled by the host at init

static __device__ const int kMaxHuffTable[23] = {256, 402, 436, 468, 500, 534, 566, 598, 630, 662, 694, 726,
                                                 758, 790, 822, 854, 886, 920, 952, 984, 1016, 1048, 1080};
static __device__ const uint8_t kCodeLenOrder[18] = {1, 2, 3, 4, 0, 5, 17, 6, 16, 7, 8, 9, 10, 11, 12, 13, 14, 15};
static __device__ const int kFixedCL[16] = {0x020000, 0x020004, 0x020003, 0x030002, 0x020000, 0x020004,
                                            0x020003, 0x040001, 0x020000, 0x020004, 0x020003, 0x030002,
                                            0x020000, 0x020004, 0x020003, 0x040005};
static __device__ const int kBlockLenOff[26] = {1, 5, 9, 13, 17, 25, 33, 41, 49, 65, 81, 97, 113,
                                                145, 177, 209, 241, 305, 369, 497, 753, 1265, 2289, 4337, 8433, 16625};
static __device__ const int8_t kBlockLenBits[26] = {2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 7, 8, 9, 10, 11, 12, 13, 24};

enum : int {
  ST_INITED = 1, ST_BLOCK_START = 2, ST_COMPRESSED_BLOCK_START = 3, ST_MAIN_LOOP = 4, ST_READ_METADATA = 5,
  ST_COPY_UNCOMPRESSED = 6, ST_INSERT_LOOP = 7, ST_COPY_LOOP = 8, ST_USE_DICTIONARY = 9, ST_FINISHED = 10,
  ST_INIT_WRITE = 12, ST_WRITE = 13, ST_COPY_FROM_COMPOUND = 14
};

constexpr int kBlockTreesCap = 3091;   // engine.ts:163 Int32Array(3091)

// LDS working set of one stream (one wave): the state below (~14 KiB) plus a table area
// declared by the kernel itself: 12,224 entries in the batch build (40 KiB per stream, four
// streams per CU), 68,096 in the one-per-CU build a call with few streams gets, which also
// keeps the block-type trees in LDS -- so a foreign stream's large prefix-code set (native
// brotli's q11 fonts: 142 literal codes in a metablock) stays in LDS.  (The table area is
// static in both builds: a dynamically sized one made the batch decode 14 % slower, 179 vs
// 157 ms on C4.)  A metablock's tables are built in HBM scratch (packed, exact sizes) and,
// when they fit, copied into the table area as 16-bit entries (nbits << 12 |
// symbol-or-subtable-offset), tree roots resolved to absolute indices.
constexpr int kLdsTab = 12224;   // the batch build's table area (4 streams per CU)
constexpr int kLdsTabBig = 68096;   // the one-stream-per-CU build's

typedef __attribute__((address_space(1))) uint8_t GU8;          // HBM
typedef const __attribute__((address_space(1))) int32_t GI32;
typedef const __attribute__((address_space(3))) uint8_t LU8;    // LDS
typedef const __attribute__((address_space(3))) int32_t LI32;
typedef const __attribute__((address_space(3))) uint16_t LU16;

struct Lds {
  uint8_t win[4160 + 64];    // byteBuffer (4160) + read slack
  uint8_t lens[1080];        // code lengths scratch
  uint16_t sorted[1080];
  int32_t cl_table[33];
  int32_t ctx_tree_base[64];
  uint8_t ctx_lut[512];        // the current literal context mode's slice of the RFC lookup table
  uint8_t mtf[256];
  uint16_t ctx_root[2048];     // (lut1[p2] << 8 | p1) -> root of the literal tree (16-bit tables)
  // part mode (parts.h): the 64 parts before this one -- lane l <-> part pidx - 1 - l: their
  // output ranges and the progress last acquired from them
  int part_lo[64], part_hi[64], part_seen[64];
};

struct Dec {
  // input
  const uint8_t *in;
  uint64_t in_len, in_off;
  uint32_t acc;
  int bo, ho, tail, eos;
  // state
  int running, next_running;
  uint8_t *ring;
  int ring_cap, ring_size, max_ring, max_back, max_dist, expected_total, pos;
  int mbl, input_end, is_uncompressed, is_metadata;
  int lit_blen, n_lit_types, cmd_blen, n_cmd_types, dist_blen, n_dist_types;
  int rings[10], dist_rb_idx;
  int32_t *lit_group, *cmd_group, *dist_group;   // HBM scratch, packed
  int32_t *tab_hbm;
  uint16_t *tab_lds;       // the 16-bit copy of the tables: the kernel's table area
  int tab16, cmd_base, dist_base;   // tables in LDS; where the command / distance groups start there
  int tab_cap;             // entries of the kernel's LDS table area
  int32_t *bt;             // block-type and block-count trees (HBM scratch, cold)
  uint8_t *ring_scratch;   // the block's HBM ring
  int direct;              // ring == out: a single-metablock stream decodes in place
  uint8_t *ctx_modes, *ctx_map, *dist_ctx_map;   // HBM scratch
  int trivial_lit_ctx, lit_tree_idx, cmd_tree_idx;
  int j, insert_len, copy_len, dist_code, distance;
  int ctx_map_slice, dist_ctx_map_slice, clo1, clo2;
  int npostfix, ndirect;
  // output (virtual 16 KiB..4 MiB chunks of the reference's unknown-size mode)
  uint8_t *out;
  int64_t out_cap, out_flushed, chunk_start, chunk_size;
  int known_size;
  int rb_written, rb_ready;
  // compound dictionary
  const uint8_t *cd;
  int cd_total, cd_br_offset, cd_br_length, cd_br_copied, cd_br_index;
  // input position of win[0] (absolute bit position = (win_base + 2 ho) * 8 - 32 + bo)
  int64_t win_base;
  // the current metablock: header bit offset, output position, length (part checks)
  int64_t mb_bit;
  int mb_pos, mb_len;
  // part mode: [part_start, part_end) of the output, progress publishing, the stream's
  // progress words (part_end = INT_MAX: whole-stream mode)
  int part, part_start, part_end, pub_next, pidx, cover_lo;
#ifdef MIB_PROF
  int pidx_g;
#endif
  int pctx;              // part mode: the two output bytes before part_start (p1 | p2 << 8, from the entry)
  uint64_t *prog;
  const int64_t *ppos;   // the stream's part start positions (+ its total at [nparts])
  Lds *l;
  uint64_t guard, guard_limit;
};

// The decoder state lives in LDS (one copy per wave): loads from it are uniform (scalar
// after readfirstlane) and, unlike a private-memory struct, never share a counter with the
// outstanding ring stores.
typedef __attribute__((address_space(3))) Dec DecS;
#define LANE ((int)threadIdx.x)
static_assert(sizeof(Lds) + sizeof(Dec) + 2 * kLdsTab <= 163840 / 4, "four streams per CU");
static_assert(sizeof(Lds) + sizeof(Dec) + 2 * kLdsTabBig + 4 * (kBlockTreesCap + 1) <= 163840 - 1024, "one stream per CU");
constexpr uint64_t kPartFailed = ~0ull;   // a part's progress word when it failed

// One stream per workgroup (one wave): the LDS working set lives at file scope, so the hot
// loop addresses it with constant offsets instead of pointer registers.
__shared__ Lds g_lds;

__shared__ Dec g_dec;   // the decoder state: LDS, so that it is wave-uniform and never waits on HBM stores
// fast_loop: the source bytes of copies in flight, by LDS-DMA.  global_load_lds_ubyte writes
// lane l's byte zero-extended to the DWORD at base + 4 l (probed on the MI355X:
// scripts/probe/glds_probe.hip), so a slot is 64 dwords; kCopyQ slots, used round robin.
constexpr int kCopyQ = 4;
__shared__ uint32_t g_cp[kCopyQ][64];
__device__ __forceinline__ uint32_t lds_addr(const __attribute__((address_space(3))) void *p) {
  return (uint32_t)(uintptr_t)p;
}
__device__ __forceinline__ uint32_t lshl1_add(uint32_t a, uint32_t b) {   // a * 2 + b, one VALU op
  uint32_t r;
  asm("v_lshl_add_u32 %0, %1, 1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// fast_loop's context-modelled literals: the chain in VGPRs (1) or through SGPRs (0, A/B builds)
#ifndef MIB_VLIT
#define MIB_VLIT 1
#endif
constexpr bool kVlit = MIB_VLIT;
// fast_loop's one-code literals: 64 entries decoded at once and walked (1), or the chain (0)
#ifndef MIB_SPECLIT
#define MIB_SPECLIT 1
#endif
constexpr bool kSpecLit = MIB_SPECLIT;

#define ERR(s, c) ((s).running = (s).running >= 0 ? (c) : (s).running, (c))

#ifdef MIB_PROF   // timing experiment: cycles in command / literal / distance / copy, literal and command counts
__device__ unsigned long long g_prof[16];   // + metablocks with LDS / HBM tables
// per part (decode_parts_kernel): start / end clock, cycles in part_wait, part_wait calls, spins,
// header done clock, commands (unused), the wave's hardware id
constexpr int kPartProfMax = 8192;
__device__ unsigned long long g_part_prof[kPartProfMax * 8];
// metablock headers: cycles in partitions + modes, context maps, literal / command / distance
// groups, the LDS copy; headers, literal trees, read_code_lengths cycles, build_table cycles
__device__ unsigned long long g_hdr_prof[16];
#define HMARK(k)                                        \
  do {                                                  \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    if (LANE == 0) atomicAdd(&g_hdr_prof[k], t_ - ht0); \
    ht0 = t_;                                           \
  } while (0)
#else
#define HMARK(k) do {} while (0)
#endif

// A block is one wave: a wave's LDS and global accesses are performed in order, so the
// lanes only need a compiler fence at wavefront scope between dependent steps.  (A
// workgroup barrier would also wait for every outstanding ring store, once per command.)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// lane `lane` of v takes the (wave-uniform) value x: one v_writelane_b32 (a compare and a
// select per literal before)
__device__ __forceinline__ uint32_t write_lane(uint32_t v, uint32_t x, uint32_t lane) {
  // The lane select goes through m0 (two SGPR operands would break the constant-bus limit).
  // m0 is an input operand ("{m0}"), so the compiler itself loads it and knows its value is
  // gone: the LDS-DMA below sets m0 to its LDS address, and m0 as a clobber is a reserved
  // register the compiler does not promise to restore (clang warns, and a hoisted m0 would
  // send a copy's bytes to the wrong LDS words).
  const uint32_t xs = (uint32_t)__builtin_amdgcn_readfirstlane((int)x), ls = (uint32_t)__builtin_amdgcn_readfirstlane((int)lane);
  asm volatile("v_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(xs), "{m0}"(ls));
  return v;
}
// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 3] (the immediate is part of the encoding)
__device__ __forceinline__ void wait_vm(int n) {
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
}

// ---------------------------------------------------------------- bit reader
__device__ __forceinline__ uint32_t half_at(const DecS &s, int h) {
  if (h < 0 || h >= 2080) return 0;   // Int16Array(2080): undefined -> 0
  return (uint32_t)s.l->win[2 * h] | ((uint32_t)s.l->win[2 * h + 1] << 8);
}
__device__ __forceinline__ void fill16(DecS &s) {
  if (s.bo >= 16) {
    s.acc = (half_at(s, s.ho++) << 16) | (s.acc >> 16);
    s.bo -= 16;
  }
}
__device__ __forceinline__ void force16(DecS &s) {
  s.acc = (half_at(s, s.ho++) << 16) | (s.acc >> 16);
  s.bo -= 16;
}
__device__ __forceinline__ uint32_t peek(const DecS &s) { return s.acc >> (s.bo & 31); }
__device__ __forceinline__ int bits(DecS &s, int n) {
  int v = (int)(peek(s) & ((1u << n) - 1u));
  s.bo += n;
  return v;
}
__device__ __forceinline__ int many_bits(DecS &s, int n) {
  int lo = bits(s, 16);
  force16(s);
  return lo | (bits(s, n - 16) << 16);
}
__device__ int half_available(const DecS &s) {
  int limit = s.eos ? (s.tail + 1) >> 1 : 2048;
  return limit - s.ho;
}

// readMoreInput (engine.ts:1764-1790): LDS memmove + HBM -> LDS fill, by the whole wave.
__device__ __noinline__ int read_more_input(DecS &s) {
  if (s.eos) return half_available(s) >= -2 ? 0 : ERR(s, -16);
  int ro = s.ho << 1;
  int have = 4096 - ro;
  if (have < 0) return MIB_E_JS_RANGE_ERROR;
  uint16_t tmp[32];
  const uint16_t *w16 = reinterpret_cast<const uint16_t *>(s.l->win);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    int idx = LANE + 64 * k;
    tmp[k] = (2 * idx < have) ? w16[(ro >> 1) + idx] : 0;
  }
  wave_sync();
  uint16_t *wo = reinterpret_cast<uint16_t *>(s.l->win);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    int idx = LANE + 64 * k;
    if (2 * idx < have) wo[idx] = tmp[k];
  }
  wave_sync();
  s.ho = 0;
  s.win_base += ro;
  uint64_t avail = s.in_len - s.in_off;
  int n = (uint64_t)(4096 - have) < avail ? 4096 - have : (int)avail;
  for (int i = LANE; i < n; i += 64) s.l->win[have + i] = s.in[s.in_off + i];
  wave_sync();
  s.in_off += (uint64_t)n;
  have += n;
  if (have < 4096) {
    s.eos = 1;
    s.tail = have;
  }
  return 0;
}
#define MAYBE_REFILL(s)                       \
  do {                                        \
    if ((s).ho > 2030) {                      \
      int r_ = read_more_input(s);            \
      if (r_ < 0) return r_;                  \
    }                                         \
  } while (0)

__device__ int check_health(DecS &s, int end_of_stream) {
  if (!s.eos) return 0;
  int byte_off = (s.ho << 1) + ((s.bo + 7) >> 3) - 4;
  if (byte_off > s.tail) return ERR(s, -13);
  if (end_of_stream && byte_off != s.tail) return ERR(s, -17);
  return 0;
}
__device__ int prepare(DecS &s) {
  MAYBE_REFILL(s);
  int h = check_health(s, 0);
  if (h) return h;
  force16(s);
  force16(s);
  return 0;
}
__device__ int jump_to_byte_boundary(DecS &s) {
  int pad = (32 - s.bo) & 7;
  if (pad && bits(s, pad) != 0) return ERR(s, -5);
  return 0;
}

// ---------------------------------------------------------------- part mode (parts.h)
constexpr int kPartFail = -120;   // internal: the part cannot vouch for its bytes (stream falls back)

__device__ __forceinline__ int64_t abs_bit(const DecS &s) { return (s.win_base + 2 * (int64_t)s.ho) * 8 - 32 + s.bo; }

// The output byte at position p >= pos - 2 (a literal context byte).  A part never reads the
// bytes before its start from the output: the previous part may still be writing them; they
// come from its entry (0 before the stream start, as in the reference's zeroed ring).
__device__ __forceinline__ int ctx_byte(const DecS &s, int p, int rmask) {
  if (s.part && p < s.part_start) return p < 0 ? 0 : (s.pctx >> (8 * (s.part_start - 1 - p))) & 0xFF;
  return s.ring[p & rmask];
}

// position the bit reader at absolute bit `bit` with a fresh 4 KiB window from there
__device__ int part_seek(DecS &s, int64_t bit) {
  const int64_t byte0 = (bit >> 3) & ~1ll;
  if (byte0 < 0 || (uint64_t)byte0 > s.in_len) return kPartFail;
  s.in_off = (uint64_t)byte0;
  s.win_base = byte0 - 4096;
  s.ho = 2048;
  s.bo = 32;
  s.acc = 0;
  s.eos = 0;
  s.tail = 0;
  const int r = prepare(s);
  if (r < 0) return r;
  s.bo += (int)(bit - 8 * byte0);
  return 0;
}

// All output bytes below pos are stored: publish pos (every storing lane drains, one
// agent-scope release, then the flag -- MI355X_MICROARCH.md "Valid forms").
__device__ __noinline__ void part_publish(int pos) {
  DecS &s = *(DecS *)&g_dec;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (LANE == 0) __hip_atomic_store(s.prog + s.pidx, (uint64_t)pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  s.pub_next = pos + (int)kPartPublish;
}
__device__ __noinline__ void part_fail() {
  DecS &s = *(DecS *)&g_dec;
  if (LANE == 0) __hip_atomic_store(s.prog + s.pidx, kPartFailed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// bytes [a, b) of earlier parts (a < b <= part_start) are readable once every part
// overlapping them has published at least min(b, its end): lane l checks part pidx - 1 - l
// against the progress this wave last acquired; parts further back are polled directly.
__device__ __forceinline__ bool part_ready_near(int a, int b, int lo, int hi, int seen, int cover_lo) {
  const bool ok = hi <= a || lo >= b || seen >= (b < hi ? b : hi);
  return a >= cover_lo && __all(ok);
}
__device__ __noinline__ int part_wait(int a, int b) {
  DecS &s = *(DecS *)&g_dec;
  const int lane = LANE, pidx = s.pidx;
  const int64_t *ppos = s.ppos;
  const int lo = g_lds.part_lo[lane], hi = g_lds.part_hi[lane];
  const int cover_lo = s.cover_lo;
#ifdef MIB_PROF
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
  for (uint32_t spin = 0;; spin++) {
    const int w = pidx - 1 - lane;
    const uint64_t v = w >= 0 ? __hip_atomic_load(s.prog + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    if (__any(v == kPartFailed)) return kPartFail;
    const int seen = (int)(v < 0x7FFFFFFFull ? v : 0x7FFFFFFFull);
    g_lds.part_seen[lane] = seen;
    bool ok = hi <= a || lo >= b || seen >= (b < hi ? b : hi);
    // parts beyond the 64 nearest: polled one by one (lane 0), from the nearest down
    if (a < cover_lo) {
      int far = 1;   // 1 ready, 0 not yet, -1 failed
      if (lane == 0) {
        for (int q = pidx - 65; q >= 0 && ppos[q + 1] > a; q--) {
          const int e = (int)ppos[q + 1];
          const uint64_t pv = __hip_atomic_load(s.prog + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (pv == kPartFailed || (int64_t)pv < (b < e ? b : e)) {
            far = pv == kPartFailed ? -1 : 0;
            break;
          }
        }
      }
      far = __shfl(far, 0);
      if (far < 0) return kPartFail;
      ok = ok && far > 0;
    }
    if (__all(ok)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // this CU's L1 drops what it held
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wave_sync();
#ifdef MIB_PROF
      if (lane == 0 && s.pidx_g < kPartProfMax) {
        unsigned long long *q = g_part_prof + 8 * s.pidx_g;
        q[2] += __builtin_amdgcn_s_memtime() - t0;
        q[3] += 1;
        q[4] += spin;
      }
#endif
      return 0;
    }
    if (spin > (1u << 24)) return kPartFail;   // (bounded: a part never waits on a later one)
    __builtin_amdgcn_s_sleep(4);
  }
}

// ---------------------------------------------------------------- Huffman tables (engine.ts:1677-1762)
__device__ int next_key(int key, int len) {
  int step = 1 << (len - 1);
  while (key & step) step >>= 1;
  return (key & (step - 1)) + step;
}
// group[off + p] = item for p = end - step, end - 2 step, ..., 0 ; lanes split the writes
__device__ __forceinline__ void replicate(const DecS &s, int32_t *g, int cap, int off, int step, int end, int item) {
  int n = end / step;
  for (int k = LANE; k < n; k += 64) {
    int i = off + k * step;
    if (i < cap) g[i] = item;
  }
}
// The per-length counts and the length-sorted symbol list by the wave (15 ballots per 64
// symbols); count[] goes to LDS scratch in ctx_root, which build_ctx_tree_base rebuilds after
// every metablock header (the private count[] / offset[] arrays, indexed by code length, were
// scratch memory: a scratch round trip per symbol, twice, in every lane).
template <class L>
__device__ int build_table(DecS &s, int32_t *group, int cap, int idx, int root, const L *lens, int nsym) {
  int toff = group[idx];
  uint32_t cnt = 0;   // lane l (1..15): symbols of length l
  for (int c0 = 0; c0 < nsym; c0 += 64) {
    const int i = c0 + LANE;
    const int l = i < nsym ? (int)lens[i] : 0;
#pragma unroll
    for (int ll = 1; ll < 16; ll++) {
      const uint64_t m = __ballot(l == ll);
      cnt += LANE == ll ? (uint32_t)__popcll(m) : 0u;
    }
  }
  uint32_t off = 0, run = 0;   // lane l: the first slot of length l in sorted
#pragma unroll
  for (int ll = 1; ll < 16; ll++) {
    off = LANE == ll ? run : off;
    run += (uint32_t)__shfl((int)cnt, ll);
  }
  const int nonzero = (int)run;
  uint16_t *sorted = s.l->sorted;
  for (int c0 = 0; c0 < nsym; c0 += 64) {
    const int i = c0 + LANE;
    const int l = i < nsym ? (int)lens[i] : 0;
    uint32_t pos = 0;
#pragma unroll
    for (int ll = 1; ll < 16; ll++) {
      const uint64_t m = __ballot(l == ll);
      const uint32_t base = (uint32_t)__shfl((int)off, ll);
      if (l == ll) pos = base + (uint32_t)__popcll(m & ((1ull << LANE) - 1));
      off += LANE == ll ? (uint32_t)__popcll(m) : 0u;
    }
    if (l) sorted[pos] = (uint16_t)i;
  }
  int *count = reinterpret_cast<int *>(s.l->ctx_root);
  if (LANE < 16) count[LANE] = LANE ? (int)cnt : 0;
  wave_sync();
  int tbits = root, tsize = 1 << tbits, total = tsize;
  if (nonzero == 1) {
    replicate(s, group, cap, toff, 1, total, sorted[0]);
    wave_sync();
    return total;
  }
  // Root-level entries, a symbol per lane: the canonical code of the i-th symbol in sorted
  // order is first[l] + (i - start[l]) (first[l + 1] = (first[l] + count[l]) << 1), and its
  // table key is that code reversed in l bits -- the key the reference's serial nextKey walk
  // (engine.ts:1677-1762) reaches at it.  (Serially: one dependent step per symbol.)
  uint32_t first_l = 0, start_l = 0;   // lane l: first[l], start[l]
  int nroot = 0;
  {
    uint32_t code = 0, start = 0;
    for (int l = 1; l < 16; l++) {
      const uint32_t c = (uint32_t)__shfl((int)cnt, l);
      first_l = LANE == l ? code : first_l;
      start_l = LANE == l ? start : start_l;
      code = (code + c) << 1;
      start += c;
      if (l == root) nroot = (int)start;
    }
  }
  auto key_of = [&](int i, int l) -> int {   // (every lane calls it: the shuffles need all)
    const uint32_t f = (uint32_t)__shfl((int)first_l, l), st = (uint32_t)__shfl((int)start_l, l);
    return l ? (int)(__builtin_bitreverse32(f + (uint32_t)i - st) >> (32 - l)) : 0;
  };
  for (int c0 = 0; c0 < nroot; c0 += 64) {
    const int i = c0 + LANE;
    const int sy = i < nroot ? (int)sorted[i] : 0;
    const int l = i < nroot ? (int)lens[sy] : 0;
    const int k0 = key_of(i, l);
    if (i < nroot)
      for (int k = k0; k < tsize; k += 1 << l)
        if (toff + k < cap) group[toff + k] = (l << 16) | sy;
  }
  int key = 0, sym = nroot, step = 1 << root;
  if (nroot < nonzero) {   // the walk of the longer codes starts at the first of them
    const int l = (int)lens[sorted[nroot]];
    key = __builtin_amdgcn_readfirstlane(key_of(nroot, l));
  }
  wave_sync();
  int mask = total - 1, low = -1, cur = toff;
  step = 1;
  for (int l = root + 1; l <= 15; l++) {
    step <<= 1;
    for (; count[l] > 0; count[l]--) {
      if ((key & mask) != low) {
        cur += tsize;
        // nextTableBitSize
        int b = l, left = 1 << (b - root);
        while (b < 15) {
          left -= count[b];
          if (left <= 0) break;
          b++;
          left <<= 1;
        }
        tbits = b - root;
        tsize = 1 << tbits;
        total += tsize;
        low = key & mask;
        if (LANE == 0 && toff + low < cap) group[toff + low] = ((tbits + root) << 16) | (cur - toff - low);
      }
      replicate(s, group, cap, cur + (key >> root), step, tsize, ((l - root) << 16) | sorted[sym++]);
      key = next_key(key, l);
    }
  }
  wave_sync();
  return total;
}
__device__ __forceinline__ int read_symbol(DecS &s, const int32_t *g, int cap, int idx) {
  int off = g[idx];
  uint32_t v = peek(s);
  off += (int)(v & 0xFF);
  int e0 = off < cap ? g[off] : 0;
  int nb = e0 >> 16, sym = e0 & 0xFFFF;
  if (nb <= 8) {
    s.bo += nb;
    return sym;
  }
  off += sym;
  off += (int)((v & ((1u << nb) - 1u)) >> 8);
  int e1 = off < cap ? g[off] : 0;
  s.bo += (e1 >> 16) + 8;
  return e1 & 0xFFFF;
}
constexpr int kNoCap = 1 << 30;

__device__ int read_code_lengths(DecS &s, const int *cl_lens, int nsym, uint8_t *lens) {   // engine.ts:305-369
  int sym = 0, prev = 8, repeat = 0, repeat_len = 0, space = 32768;
  int32_t *table = s.l->cl_table;
  if (LANE == 0) table[32] = 0;
  wave_sync();
  build_table(s, table, kNoCap, 32, 5, cl_lens, 18);
  // The reader's (acc, bo, ho) in registers and the 32-entry table in lanes (lane p: entry p):
  // a symbol is a register shift and a readlane, not a chain of LDS round trips through the
  // state (a metablock header of 24 literal and 4 command codes: 2.5 M cycles in here before).
  const int tab = table[LANE & 31];
  uint32_t acc = s.acc;
  int bo = s.bo, ho = s.ho;
  const uint8_t *win = s.l->win;
  auto fill = [&]() {
    if (bo >= 16) {
      const uint32_t h = (ho >= 0 && ho < 2080) ? ((uint32_t)win[2 * ho] | ((uint32_t)win[2 * ho + 1] << 8)) : 0u;
      ho++;
      acc = (h << 16) | (acc >> 16);
      bo -= 16;
    }
  };
  int rc = 0;
  while (sym < nsym && space > 0) {
    if (ho > 2030) {   // MAYBE_REFILL with the state written back around it
      s.acc = acc;
      s.bo = bo;
      s.ho = ho;
      wave_sync();
      rc = read_more_input(s);
      if (rc < 0) return rc;
      acc = s.acc;
      bo = s.bo;
      ho = s.ho;
    }
    fill();
    const int p = (int)((acc >> (bo & 31)) & 31);
    const int e = __builtin_amdgcn_readlane(tab, p);
    bo += e >> 16;
    const int len = e & 0xFFFF;
    if (len < 16) {
      repeat = 0;
      if (LANE == 0) lens[sym] = (uint8_t)len;
      sym++;
      if (len) {
        prev = len;
        space -= 32768 >> len;
      }
    } else {
      const int eb = len - 14, new_len = len == 16 ? prev : 0;
      if (repeat_len != new_len) {
        repeat = 0;
        repeat_len = new_len;
      }
      const int old = repeat;
      if (repeat > 0) {
        repeat -= 2;
        repeat <<= eb;
      }
      fill();
      repeat += (int)((acc >> (bo & 31)) & ((1u << eb) - 1u)) + 3;
      bo += eb;
      const int delta = repeat - old;
      if (sym + delta > nsym) {
        rc = ERR(s, -2);
        break;
      }
      for (int k = LANE; k < delta; k += 64) lens[sym + k] = (uint8_t)repeat_len;
      sym += delta;
      if (repeat_len) space -= delta << (15 - repeat_len);
    }
  }
  s.acc = acc;
  s.bo = bo;
  s.ho = ho;
  wave_sync();
  if (rc < 0) return rc;
  if (space != 0) return ERR(s, -18);
  for (int k = sym + LANE; k < nsym; k += 64) lens[k] = 0;
  wave_sync();
  return 0;
}

__device__ int read_huffman_code(DecS &s, int amax, int alimit, int32_t *group, int cap, int idx) {   // :370-470
  uint8_t *lens = s.l->lens;
  MAYBE_REFILL(s);
  fill16(s);
  int kind = bits(s, 2);
  for (int k = LANE; k < alimit; k += 64) lens[k] = 0;
  wave_sync();
  if (kind == 1) {
    int syms[4];
    int maxbits = 0;
    for (int v = amax - 1; v; v >>= 1) maxbits++;
    int n = bits(s, 2) + 1;
    for (int i = 0; i < n; i++) {
      fill16(s);
      int sy = bits(s, maxbits);
      if (sy >= alimit) return ERR(s, -15);
      syms[i] = sy;
    }
    for (int i = 0; i < n - 1; i++)
      for (int k = i + 1; k < n; k++)
        if (syms[i] == syms[k]) return ERR(s, -7);
    int hid = n;
    if (n == 4) hid += bits(s, 1);
    if (LANE == 0) {
      switch (hid) {
        case 1: lens[syms[0]] = 1; break;
        case 2: lens[syms[0]] = 1; lens[syms[1]] = 1; break;
        case 3: lens[syms[0]] = 1; lens[syms[1]] = 2; lens[syms[2]] = 2; break;
        case 4: for (int i = 0; i < 4; i++) lens[syms[i]] = 2; break;
        case 5: lens[syms[0]] = 1; lens[syms[1]] = 2; lens[syms[2]] = 3; lens[syms[3]] = 3; break;
      }
    }
    wave_sync();
    return build_table(s, group, cap, idx, 8, lens, alimit);
  }
  int *cl = reinterpret_cast<int *>(s.l->ctx_root) + 32;   // (LDS scratch, see build_table)
  if (LANE < 18) cl[LANE] = 0;
  wave_sync();
  int space = 32, ncodes = 0;
  for (int i = kind; i < 18; i++) {
    int ci = kCodeLenOrder[i];
    fill16(s);
    int p = (int)(peek(s) & 15);
    s.bo += kFixedCL[p] >> 16;
    int v = kFixedCL[p] & 0xFFFF;
    cl[ci] = v;
    if (v) {
      space -= 32 >> v;
      ncodes++;
      if (space <= 0) break;
    }
  }
  if (space != 0 && ncodes != 1) return ERR(s, -4);
#ifdef MIB_PROF
  unsigned long long ht0 = __builtin_amdgcn_s_memtime();
#endif
  int r = read_code_lengths(s, cl, alimit, lens);
  if (r < 0) return r;
  HMARK(7);
  r = build_table(s, group, cap, idx, 8, lens, alimit);
  HMARK(8);
  return r;
}

__device__ int decode_var_len_byte(DecS &s) {
  fill16(s);
  if (bits(s, 1)) {
    int n = bits(s, 3);
    if (n == 0) return 1;
    return bits(s, n) + (1 << n);
  }
  return 0;
}

__device__ int decode_context_map(DecS &s, int size, uint8_t *map, int32_t *table_scratch) {   // :488-558
  MAYBE_REFILL(s);
  int ntrees = decode_var_len_byte(s) + 1;
  if (ntrees == 1) {
    for (int k = LANE; k < size; k += 64) map[k] = 0;
    wave_sync();
    return ntrees;
  }
  fill16(s);
  int rle_max = 0;
  if (bits(s, 1)) rle_max = bits(s, 4) + 1;
  int asize = ntrees + rle_max;
  int tsize = kMaxHuffTable[(asize + 31) >> 5];
  int32_t *table = table_scratch;
  if (LANE == 0) table[tsize] = 0;
  wave_sync();
  int r = read_huffman_code(s, asize, asize, table, kNoCap, tsize);
  if (r < 0) return r;
  int i = 0;
  while (i < size) {
    MAYBE_REFILL(s);
    fill16(s);
    int code = read_symbol(s, table, kNoCap, tsize);
    if (code == 0) {
      if (LANE == 0) map[i] = 0;
      i++;
    } else if (code <= rle_max) {
      fill16(s);
      int reps = (1 << code) + bits(s, code);
      if (i + reps > size) return ERR(s, -3);
      for (int k = LANE; k < reps; k += 64) map[i + k] = 0;
      i += reps;
    } else {
      if (LANE == 0) map[i] = (uint8_t)(code - rle_max);
      i++;
    }
  }
  wave_sync();
  fill16(s);
  if (bits(s, 1) == 1) {   // inverse move-to-front, lane 0 (rare, small)
    if (LANE == 0) {
      uint8_t *mtf = s.l->mtf;
      for (int k = 0; k < 256; k++) mtf[k] = (uint8_t)k;
      for (int k = 0; k < size; k++) {
        int index = map[k];
        int v = mtf[index];
        map[k] = (uint8_t)v;
        for (int q = index; q > 0; q--) mtf[q] = mtf[q - 1];
        mtf[0] = (uint8_t)v;
      }
    }
    wave_sync();
  }
  return ntrees;
}

__device__ int read_block_length(DecS &s, const int32_t *g, int idx) {
  fill16(s);
  int code = read_symbol(s, g, kBlockTreesCap, idx);
  int n = kBlockLenBits[code];
  fill16(s);
  return kBlockLenOff[code] + (n <= 16 ? bits(s, n) : many_bits(s, n));
}
__device__ __noinline__ int decode_block_type_and_length(DecS &s, int tree_type, int ntypes) {   // :559-580
  int off = 4 + tree_type * 2;
  fill16(s);
  int bt = read_symbol(s, s.bt, kBlockTreesCap, 2 * tree_type);
  int len = read_block_length(s, s.bt, 2 * tree_type + 1);
  if (bt == 1) bt = s.rings[off + 1] + 1;
  else if (bt == 0) bt = s.rings[off];
  else bt -= 2;
  if (bt >= ntypes) bt -= ntypes;
  s.rings[off] = s.rings[off + 1];
  s.rings[off + 1] = bt;
  return len;
}
__device__ __noinline__ void build_ctx_tree_base(DecS &s) {
  for (int k = LANE; k < 512; k += 64) s.l->ctx_lut[k] = kRfcContextLut[s.clo1 + k];
  const int tree = s.ctx_map[s.ctx_map_slice + LANE];
  if (s.tab16) {
    // lut0[p1] | lut1[p2] with lut1 < 8 in every mode: one (p1, lut1[p2]) -> root table
    const int root = s.tab_lds[tree];   // the literal group starts at 0
    wave_sync();
    for (int k = LANE; k < 2048; k += 64) s.l->ctx_root[k] = (uint16_t)__shfl(root, s.l->ctx_lut[k & 255] | (k >> 8));
  } else {
    s.l->ctx_tree_base[LANE] = s.lit_group[tree];
  }
  wave_sync();
}
__device__ __noinline__ void lit_block_switch(DecS &s) {
  s.lit_blen = decode_block_type_and_length(s, 0, s.n_lit_types);
  int t = s.rings[5];
  s.ctx_map_slice = t << 6;
  s.lit_tree_idx = s.ctx_map[s.ctx_map_slice];
  int mode = s.ctx_modes[t];
  s.clo1 = mode << 9;
  s.clo2 = s.clo1 + 256;
}

// back to the block's own ring: its content so far is the output's first ring_size bytes
__device__ void leave_direct(DecS &s) {
  const int n = s.ring_size + 37;
  for (int k = LANE; k < n; k += 64) s.ring_scratch[k] = k < s.out_cap ? s.out[k] : 0;
  wave_sync();
  s.ring = s.ring_scratch;
  s.direct = 0;
}

__device__ void maybe_realloc_ring(DecS &s) {   // :608-630 (the scratch slice is max-sized; copy semantics kept)
  int new_size = s.max_ring;
  if (new_size > s.expected_total) {
    int minimal = s.expected_total;
    while ((new_size >> 1) > minimal) new_size >>= 1;
    if (!s.input_end && new_size < 16384 && s.max_ring >= 16384) new_size = 16384;
  }
  if (new_size <= s.ring_size) return;
  // A stream announced as one final metablock whose ring fits the output buffer decodes
  // straight into the output: the ring's bytes [0, pos) are then exactly the output's,
  // so every flush is an identity and the ring -> output copy disappears.
  if (s.ring_size == 0 && s.input_end && s.out_flushed == 0 && (int64_t)new_size + 37 + 64 <= s.out_cap) {
    s.ring = s.out;
    s.direct = 1;
  } else if (s.direct && (int64_t)new_size + 37 + 64 > s.out_cap) {
    leave_direct(s);
  }
  // a fresh Uint8Array: bytes beyond the old size are zero
  for (int k = s.ring_size + LANE; k < new_size + 37; k += 64) s.ring[k] = 0;
  wave_sync();
  s.ring_cap = new_size + 37;
  s.ring_size = new_size;
}

__device__ int decode_mb_length(DecS &s) {   // :204-256
  fill16(s);
  s.input_end = bits(s, 1);
  s.mbl = 0;
  s.is_uncompressed = 0;
  s.is_metadata = 0;
  if (s.input_end && bits(s, 1)) return 0;
  int nibbles = bits(s, 2) + 4;
  if (nibbles == 7) {
    s.is_metadata = 1;
    if (bits(s, 1)) return ERR(s, -6);
    int nbytes = bits(s, 2);
    if (nbytes == 0) return 0;
    for (int i = 0; i < nbytes; i++) {
      fill16(s);
      int b = bits(s, 8);
      if (b == 0 && i + 1 == nbytes && nbytes > 1) return ERR(s, -8);
      s.mbl += b << (i * 8);
    }
  } else {
    for (int i = 0; i < nibbles; i++) {
      fill16(s);
      int b = bits(s, 4);
      if (b == 0 && i + 1 == nibbles && nibbles > 4) return ERR(s, -8);
      s.mbl += b << (i * 4);
    }
  }
  s.mbl++;
  if (!s.input_end) s.is_uncompressed = bits(s, 1);
  return 0;
}

__device__ int read_next_mb_header(DecS &s) {   // :631-678
  if (s.input_end) {
    s.next_running = ST_FINISHED;
    s.running = ST_INIT_WRITE;
    return 0;
  }
  MAYBE_REFILL(s);
  const int64_t hbit = abs_bit(s);
  int r = decode_mb_length(s);
  if (r < 0) return r;
  s.mb_bit = hbit;
  s.mb_pos = s.pos;
  s.mb_len = s.mbl;
  if (s.mbl == 0 && !s.is_metadata) return 0;
  if (s.is_uncompressed || s.is_metadata) {
    r = jump_to_byte_boundary(s);
    if (r < 0) return r;
    s.running = s.is_metadata ? ST_READ_METADATA : ST_COPY_UNCOMPRESSED;
  } else {
    s.running = ST_COMPRESSED_BLOCK_START;
  }
  if (s.is_metadata) return 0;
  s.expected_total += s.mbl;
  if (s.expected_total > (1 << 30)) s.expected_total = 1 << 30;
  if (s.ring_size < s.max_ring) maybe_realloc_ring(s);
  return 0;
}

__device__ int read_partition(DecS &s, int tt, int ntypes) {   // :679-704
  int32_t *bt = s.bt;
  int off = bt[2 * tt];
  if (ntypes <= 1) {
    wave_sync();
    if (LANE == 0) {
      bt[2 * tt + 1] = off;
      bt[2 * tt + 2] = off;
    }
    wave_sync();
    return 1 << 28;
  }
  int r = read_huffman_code(s, ntypes + 2, ntypes + 2, bt, kBlockTreesCap, 2 * tt);
  if (r < 0) return r;
  off += r;
  if (LANE == 0) bt[2 * tt + 1] = off;
  wave_sync();
  r = read_huffman_code(s, 26, 26, bt, kBlockTreesCap, 2 * tt + 1);
  if (r < 0) return r;
  off += r;
  if (LANE == 0) bt[2 * tt + 2] = off;
  wave_sync();
  return read_block_length(s, bt, 2 * tt + 1);
}

__device__ int decode_tree_group(DecS &s, int amax, int alimit, int n, int32_t *group) {
  int next = n;
  for (int i = 0; i < n; i++) {
    if (LANE == 0) group[i] = next;
    wave_sync();
    int r = read_huffman_code(s, amax, alimit, group, kNoCap, i);
    if (r < 0) return r;
    next += r;
  }
  return next;   // the group's size in ints: its n roots and its tables
}

__device__ int read_codes_and_maps(DecS &s, int8_t *dist_extra, int32_t *dist_offset, int32_t *ctxmap_table) {
  int r;
#ifdef MIB_PROF
  unsigned long long ht0 = __builtin_amdgcn_s_memtime();
#endif
  s.n_lit_types = decode_var_len_byte(s) + 1;
  if ((r = read_partition(s, 0, s.n_lit_types)) < 0) return r;
  s.lit_blen = r;
  s.n_cmd_types = decode_var_len_byte(s) + 1;
  if ((r = read_partition(s, 1, s.n_cmd_types)) < 0) return r;
  s.cmd_blen = r;
  s.n_dist_types = decode_var_len_byte(s) + 1;
  if ((r = read_partition(s, 2, s.n_dist_types)) < 0) return r;
  s.dist_blen = r;
  MAYBE_REFILL(s);
  fill16(s);
  s.npostfix = bits(s, 2);
  s.ndirect = bits(s, 4) << s.npostfix;
  int i = 0;
  while (i < s.n_lit_types) {
    int lim = i + 96 < s.n_lit_types ? i + 96 : s.n_lit_types;
    while (i < lim) {
      fill16(s);
      int m = bits(s, 2);
      if (LANE == 0) s.ctx_modes[i] = (uint8_t)m;
      i++;
    }
    MAYBE_REFILL(s);
  }
  int cml = s.n_lit_types << 6;
  HMARK(0);
  if ((r = decode_context_map(s, cml, s.ctx_map, ctxmap_table)) < 0) return r;
  int nlit_trees = r;
  int nontrivial = 0;
  for (int k = LANE; k < cml; k += 64)
    if (s.ctx_map[k] != (k >> 6)) nontrivial = 1;
  s.trivial_lit_ctx = __any(nontrivial) ? 0 : 1;
  if ((r = decode_context_map(s, s.n_dist_types << 2, s.dist_ctx_map, ctxmap_table)) < 0) return r;
  int ndist_trees = r;
  HMARK(1);
  // groups live back to back: literal, command, distance.  A metablock with few prefix
  // codes (the common case: one tree per alphabet) gets them in LDS, so every symbol
  // lookup is an LDS read instead of a dependent HBM load.
  s.lit_group = s.tab_hbm;
  if ((r = decode_tree_group(s, 256, 256, nlit_trees, s.lit_group)) < 0) return r;
  HMARK(2);
#ifdef MIB_PROF
  if (LANE == 0) {
    atomicAdd(&g_hdr_prof[5], 1ull);
    atomicAdd(&g_hdr_prof[6], (unsigned long long)nlit_trees);
  }
#endif
  s.cmd_group = s.lit_group + r;
  if ((r = decode_tree_group(s, 704, 704, s.n_cmd_types, s.cmd_group)) < 0) return r;
  HMARK(3);
  s.dist_group = s.cmd_group + r;
  int dmax = 16 + s.ndirect + 2 * (24 << s.npostfix);
  if ((r = decode_tree_group(s, dmax, dmax, ndist_trees, s.dist_group)) < 0) return r;
  HMARK(4);
  // tables that fit go to LDS as 16-bit entries, roots made absolute
  const int cmd_base = (int)(s.cmd_group - s.lit_group), dist_base = (int)(s.dist_group - s.lit_group);
  const int total = dist_base + r;
  s.tab16 = total <= s.tab_cap;
#ifdef MIB_PROF
  if (LANE == 0) atomicAdd(&g_prof[s.tab16 ? 6 : 7], 1ull);
#endif
  s.cmd_base = cmd_base;
  s.dist_base = dist_base;
  if (s.tab16) {
    const int32_t *src = s.lit_group;
    for (int k = LANE; k < total; k += 64) {
      const int v = src[k];
      int o;
      if (k < nlit_trees) o = v;
      else if (k >= cmd_base && k < cmd_base + s.n_cmd_types) o = v + cmd_base;
      else if (k >= dist_base && k < dist_base + ndist_trees) o = v + dist_base;
      else o = ((v >> 16) << 12) | (v & 0xFFF);
      s.tab_lds[k] = (uint16_t)o;
    }
    wave_sync();
  }
  // calculateDistanceLut (:705-726), lane 0
  if (LANE == 0) {
    int np = s.npostfix, nd = s.ndirect, postfix = 1 << np, b = 1, half = 0, k = 16;
    for (int q = 0; q < nd; q++) {
      dist_extra[k] = 0;
      dist_offset[k] = q + 1;
      k++;
    }
    while (k < dmax) {
      int base = nd + ((((2 + half) << b) - 4) << np) + 1;
      for (int q = 0; q < postfix; q++) {
        dist_extra[k] = (int8_t)b;
        dist_offset[k] = base + q;
        k++;
      }
      b += half;
      half ^= 1;
    }
  }
  wave_sync();
  s.ctx_map_slice = 0;
  s.dist_ctx_map_slice = 0;
  s.clo1 = s.ctx_modes[0] * 512;
  s.clo2 = s.clo1 + 256;
  build_ctx_tree_base(s);
  s.lit_tree_idx = 0;
  s.cmd_tree_idx = 0;
  s.rings[4] = 1; s.rings[5] = 0; s.rings[6] = 1; s.rings[7] = 0; s.rings[8] = 1; s.rings[9] = 0;
  HMARK(9);
  return 0;
}

// copyRawBytes (:1876-1925) into the ring
__device__ int copy_raw_bytes(DecS &s, int pos, int len) {
  if (s.bo & 7) return ERR(s, -30);
  while (s.bo != 32 && len) {
    if (LANE == 0) s.ring[pos] = (uint8_t)peek(s);
    pos++;
    s.bo += 8;
    len--;
  }
  wave_sync();
  if (!len) return 0;
  int ha = half_available(s);
  int cn = ha < (len >> 1) ? ha : (len >> 1);
  if (cn > 0) {
    int ro = s.ho << 1, delta = cn << 1;
    for (int k = LANE; k < delta; k += 64) s.ring[pos + k] = s.l->win[ro + k];
    wave_sync();
    pos += delta;
    len -= delta;
    s.ho += cn;
  }
  if (!len) return 0;
  if (half_available(s) > 0) {
    fill16(s);
    while (len) {
      if (LANE == 0) s.ring[pos] = (uint8_t)peek(s);
      pos++;
      s.bo += 8;
      len--;
    }
    wave_sync();
    return check_health(s, 0);
  }
  uint64_t avail = s.in_len - s.in_off;
  if ((uint64_t)len > avail) {   // readInput returns what is left, then 0 -> error -16
    for (uint64_t k = LANE; k < avail; k += 64) s.ring[pos + k] = s.in[s.in_off + k];
    s.in_off += avail;
    wave_sync();
    return ERR(s, -16);
  }
  for (int k = LANE; k < len; k += 64) s.ring[pos + k] = s.in[s.in_off + k];
  s.in_off += (uint64_t)len;
  wave_sync();
  return 0;
}

// write_ring (:868-879) + the reference's chunked output (:2223-2256) as one linear buffer.
// Returns 0 (space left in the current chunk), 2 (chunk / known buffer full), or NEED_SPACE.
__device__ int write_ring(DecS &s) {
  int64_t chunk_left = s.chunk_start + s.chunk_size - s.out_flushed;
  int64_t b = s.rb_ready - s.rb_written;
  int64_t n = chunk_left < b ? chunk_left : b;
  if (n > 0) {
    if (s.out_flushed + n > s.out_cap) return MIB_E_NEED_SPACE;
    uint8_t *dst = s.out + s.out_flushed;
    const uint8_t *src = s.ring + s.rb_written;
    if (dst != src) {   // (decoding in place: nothing to move)
      for (int64_t k = LANE; k < n; k += 64) dst[k] = src[k];
      wave_sync();
    }
    s.out_flushed += n;
    s.rb_written += (int)n;
  }
  return s.out_flushed < s.chunk_start + s.chunk_size ? 0 : 2;
}

// static dictionary word + RFC transform, lane 0 (engine.ts:1557-1675)
__device__ int transform_word(uint8_t *dst, int doff, int soff, int wlen, int tidx) {
  int off = doff;
  int pre = kRfcTransformTriplets[3 * tidx], type = kRfcTransformTriplets[3 * tidx + 1],
      suf = kRfcTransformTriplets[3 * tidx + 2];
  int p = kRfcPrefixSuffixHeads[pre], pe = kRfcPrefixSuffixHeads[pre + 1];
  int q = kRfcPrefixSuffixHeads[suf], qe = kRfcPrefixSuffixHeads[suf + 1];
  int omit_first = type - 11, omit_last = type;
  if (omit_first < 1 || omit_first > 9) omit_first = 0;
  if (omit_last < 1 || omit_last > 9) omit_last = 0;
  while (p != pe) dst[off++] = kRfcPrefixSuffix[p++];
  int len = wlen;
  if (omit_first > len) omit_first = len;
  int so = soff + omit_first;
  len -= omit_first;
  len -= omit_last;
  for (int i = len; i > 0; i--) dst[off++] = kDictionary[so++];
  if (type == 10 || type == 11) {
    int u = off - len;
    if (type == 10) len = 1;
    while (len > 0) {
      int c0 = dst[u];
      if (c0 < 0xC0) {
        if (c0 >= 97 && c0 <= 122) dst[u] ^= 32;
        u += 1;
        len -= 1;
      } else if (c0 < 0xE0) {
        dst[u + 1] ^= 32;
        u += 2;
        len -= 2;
      } else {
        dst[u + 2] ^= 5;
        u += 3;
        len -= 3;
      }
    }
  }
  while (q != qe) dst[off++] = kRfcPrefixSuffix[q++];
  return off - doff;
}

__device__ int use_dictionary(DecS &s, int fence) {   // :903-983
  if (s.distance > 0x7FFFFFFC) return ERR(s, -9);
  int address = s.distance - s.max_dist - 1 - s.cd_total;
  if (address < 0) {   // compound dictionary, one chunk (attachDictionaryChunk is called once)
    int a = -address - 1, length = s.copy_len;
    if (s.cd_total > a + length) return ERR(s, -9);
    s.dist_rb_idx = (s.dist_rb_idx + 1) & 3;
    s.rings[s.dist_rb_idx] = s.distance;
    s.mbl -= length;
    s.cd_br_index = 0;
    s.cd_br_offset = a;
    s.cd_br_length = length;
    s.cd_br_copied = 0;
    s.running = ST_COPY_FROM_COMPOUND;
    return 0;
  }
  int wlen = s.copy_len;
  if (wlen > 31) return ERR(s, -9);
  int shift = kRfcDictSizeBits[wlen];
  if (shift == 0) return ERR(s, -9);
  int off = (int)kRfcDictOffsets[wlen];
  int mask = (1 << shift) - 1;
  int widx = address & mask, tidx = address >> shift;
  off += widx * wlen;
  if (tidx >= RFC_NUM_TRANSFORMS) return ERR(s, -9);
  int len = 0;
  if (LANE == 0) len = transform_word(s.ring, s.pos, off, wlen, tidx);
  len = __shfl(len, 0);
  wave_sync();
  s.pos += len;
  s.mbl -= len;
  if (s.pos >= fence) {
    s.next_running = ST_MAIN_LOOP;
    s.running = ST_INIT_WRITE;
    return 0;
  }
  s.running = ST_MAIN_LOOP;
  return 0;
}

__device__ int copy_from_compound(DecS &s, int fence) {
  int pos = s.pos, orig = pos;
  while (s.cd_br_length != s.cd_br_copied) {
    int space = fence - pos;
    int clen = s.cd_br_index == 0 ? s.cd_total : 0;
    int rem = clen - s.cd_br_offset;
    int len = s.cd_br_length - s.cd_br_copied;
    if (len > rem) len = rem;
    if (len > space) len = space;
    if (s.cd_br_index >= 1) return MIB_E_JS_TYPE_ERROR;   // reads past the last chunk in JS
    for (int k = LANE; k < len; k += 64) s.ring[pos + k] = s.cd[s.cd_br_offset + k];
    wave_sync();
    pos += len;
    s.cd_br_offset += len;
    s.cd_br_copied += len;
    if (len == rem) {
      s.cd_br_index++;
      s.cd_br_offset = 0;
    }
    if (pos >= fence) break;
  }
  return pos - orig;
}

// LZ77 copy of `cl` bytes at ring position pos from distance dist (no fence crossing).
// An overlapping copy (dist < cl) repeats the dist bytes before pos, so every byte is a
// function of pre-copy data only: out[pos + j] = ring[src + j % dist]; all 64 lanes work.
__device__ void ring_copy_fast(DecS &s, int src, int cl, int dist) {
  uint8_t *r = s.ring;
  int dst = s.pos;
  if (dist >= cl) {
    for (int k = LANE; k < cl; k += 64) r[dst + k] = r[src + k];
  } else {
    int q = LANE % dist;
    int qstep = 64 % dist;
    for (int k = LANE; k < cl; k += 64) {
      r[dst + k] = r[src + q];
      q += qstep;
      if (q >= dist) q -= dist;
    }
  }
  wave_sync();
}

// The command / literal / copy loop (engine.ts:1059-1438) as a function of its own: only
// the hot state is live in it, so it stays in SGPRs (the whole state machine inlined into
// the kernel spilled ~190 SGPRs into VGPR lanes, read and written back on every command).
// Returns 0 with s.running set for the state machine, or a negative error code.
template <bool kTabLds>
__device__ __noinline__ int hot_loop(int fence_in, int rmask_in, int stop_at_boundary) {
  DecS &s = *(DecS *)&g_dec;
  const int fence = __builtin_amdgcn_readfirstlane(fence_in), rmask = __builtin_amdgcn_readfirstlane(rmask_in);
        // The command / literal / copy loop runs on registers: the bit reader, positions,
        // lengths and block counters are loaded from `s` once, saved back around every
        // cold call (refill, block switch) and on every exit.
        // Memory is addressed through address-space-typed pointers: LDS reads then wait only
        // on LDS (lgkmcnt) and never on the outstanding HBM stores of the output, which a
        // generic (flat) access would have to drain first.
        int phase = s.running;
        GU8 *ring = (GU8 *)s.ring;
        LU16 *win16 = (LU16 *)g_lds.win;
        LI32 *ctb = (LI32 *)g_lds.ctx_tree_base;
        const int ring_cap = s.ring_cap, npostfix = s.npostfix, ndirect = s.ndirect, max_back = s.max_back;
        constexpr bool tab_lds = kTabLds;   // prefix-code tables in LDS (16-bit) or HBM
        LU16 *t16 = (LU16 *)s.tab_lds;
        LU16 *croot = (LU16 *)g_lds.ctx_root;
        const int cmd_base = __builtin_amdgcn_readfirstlane(s.cmd_base), dist_base = __builtin_amdgcn_readfirstlane(s.dist_base);
        GI32 *cmd_h = (GI32 *)s.cmd_group, *dist_h = (GI32 *)s.dist_group, *lit_h = (GI32 *)s.lit_group;
        const int lane = LANE;
        const uint64_t guard_limit = s.guard_limit;
        int trivial = s.trivial_lit_ctx, lit_tree = s.lit_tree_idx;
        const int ring_size = s.ring_size;
        LU8 *clut = (LU8 *)g_lds.ctx_lut;
        const int part = __builtin_amdgcn_readfirstlane(s.part), part_end = __builtin_amdgcn_readfirstlane(s.part_end);
        const int pstart = __builtin_amdgcn_readfirstlane(s.part_start), cover_lo = __builtin_amdgcn_readfirstlane(s.cover_lo);
        // The last two output bytes (the literal context) live in registers: reading them
        // back from the ring would wait for every outstanding ring store (vmcnt is in order).
        // (part mode: absolute positions -- before the stream start the context bytes are 0;
        // the ring's last bytes would lie past the output buffer)
        int c1 = __builtin_amdgcn_readfirstlane(ctx_byte(s, s.pos - 1, rmask));
        int c2b = __builtin_amdgcn_readfirstlane(ctx_byte(s, s.pos - 2, rmask));
        int dr0, dr1, dr2, dr3, dridx;   // the distance ring (rings[0..3], dist_rb_idx)
        uint32_t acc;
        int bo, ho, pos, j, mbl, insert_len, copy_len, dist_code, distance, cmd_blen, lit_blen, dist_blen, max_dist;
        uint64_t guard;
#define U(x) __builtin_amdgcn_readfirstlane(x)   /* the decoder state is wave-uniform: keep it scalar */
#define HOT_LOAD()                                                                                      \
  do {                                                                                                  \
    acc = U(s.acc); bo = U(s.bo); ho = U(s.ho); pos = U(s.pos); j = U(s.j); mbl = U(s.mbl);             \
    insert_len = U(s.insert_len); copy_len = U(s.copy_len); dist_code = U(s.dist_code);                 \
    distance = U(s.distance); cmd_blen = U(s.cmd_blen); lit_blen = U(s.lit_blen);                       \
    dist_blen = U(s.dist_blen); max_dist = U(s.max_dist); guard = s.guard;                              \
    dr0 = U(s.rings[0]); dr1 = U(s.rings[1]); dr2 = U(s.rings[2]); dr3 = U(s.rings[3]);                 \
    dridx = U(s.dist_rb_idx); trivial = U(s.trivial_lit_ctx); lit_tree = U(s.lit_tree_idx);             \
  } while (0)
#define HOT_SAVE()                                                                                      \
  do {                                                                                                  \
    s.acc = acc; s.bo = bo; s.ho = ho; s.pos = pos; s.j = j; s.mbl = mbl; s.insert_len = insert_len;    \
    s.copy_len = copy_len; s.dist_code = dist_code; s.distance = distance; s.cmd_blen = cmd_blen;       \
    s.lit_blen = lit_blen; s.dist_blen = dist_blen; s.max_dist = max_dist; s.guard = guard;              \
    s.rings[0] = dr0; s.rings[1] = dr1; s.rings[2] = dr2; s.rings[3] = dr3; s.dist_rb_idx = dridx;       \
  } while (0)
#define LHALF(h) (((h) < 0 || (h) >= 2080) ? 0u : (uint32_t)U((int)win16[h]))
#define LFILL16()                                     \
  do {                                                \
    if (bo >= 16) {                                   \
      acc = (LHALF(ho) << 16) | (acc >> 16);          \
      ho++;                                           \
      bo -= 16;                                       \
    }                                                 \
  } while (0)
#define LREFILL()                                     \
  do {                                                \
    if (ho > 2030) {                                  \
      HOT_SAVE();                                     \
      int r_ = U(read_more_input(s));                 \
      if (r_ < 0) return r_;                          \
      HOT_LOAD();                                     \
    }                                                 \
  } while (0)
        HOT_LOAD();
        const uint64_t guard0 = guard + 1;
        auto lbits = [&](int n) -> int {
          int v = (int)((acc >> (bo & 31)) & ((1u << n) - 1u));
          bo += n;
          return v;
        };
        auto lmany = [&](int n) -> int {
          int lo = lbits(16);
          acc = (LHALF(ho) << 16) | (acc >> 16);
          ho++;
          bo -= 16;
          return lo | (lbits(n - 16) << 16);
        };
        auto dr_get = [&](int i) -> int { return i == 0 ? dr0 : i == 1 ? dr1 : i == 2 ? dr2 : dr3; };
        auto lsym16 = [&](int root) -> int {   // read_symbol on a 16-bit LDS table with an absolute root
          uint32_t v = acc >> (bo & 31);
          int off = root + (int)(v & 0xFF);
          const int e0 = U((int)t16[off]);
          const int nb = e0 >> 12;
          if (nb <= 8) {
            bo += nb;
            return e0 & 0xFFF;
          }
          off += (e0 & 0xFFF) + (int)((v & ((1u << nb) - 1u)) >> 8);
          const int e1 = U((int)t16[off]);
          bo += (e1 >> 12) + 8;
          return e1 & 0xFFF;
        };
        auto lsym = [&](auto g, int idx) -> int {   // read_symbol on registers
          int off = U(g[idx]);
          uint32_t v = acc >> (bo & 31);
          off += (int)(v & 0xFF);
          int e0 = U(g[off]);
          int nb = e0 >> 16;
          if (nb <= 8) {
            bo += nb;
            return e0 & 0xFFFF;
          }
          off += e0 & 0xFFFF;
          off += (int)((v & ((1u << nb) - 1u)) >> 8);
          int e1 = U(g[off]);
          bo += (e1 >> 16) + 8;
          return e1 & 0xFFFF;
        };
        int cmd_tree_idx = __builtin_amdgcn_readfirstlane(s.cmd_tree_idx);
        uint32_t dtrees = 0;   // the 4 distance trees of the current distance block type
        for (int q = 0; q < 4; q++) dtrees |= (uint32_t)s.dist_ctx_map[s.dist_ctx_map_slice + q] << (8 * q);
        dtrees = U(dtrees);
        // 16-bit tables: the command root and the 4 distance roots, absolute
        int cmd_root = tab_lds ? U((int)t16[cmd_base + cmd_tree_idx]) : 0;
        uint32_t droot01 = 0, droot23 = 0;
        auto dist_roots = [&]() {
          if (!tab_lds) return;
          const int r0 = t16[dist_base + (dtrees & 0xFF)], r1 = t16[dist_base + ((dtrees >> 8) & 0xFF)];
          const int r2 = t16[dist_base + ((dtrees >> 16) & 0xFF)], r3 = t16[dist_base + (dtrees >> 24)];
          droot01 = U((int)((uint32_t)r0 | ((uint32_t)r1 << 16)));
          droot23 = U((int)((uint32_t)r2 | ((uint32_t)r3 << 16)));
        };
        dist_roots();
#ifdef MIB_PROF
        uint64_t prof[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        uint64_t pt0 = __builtin_amdgcn_s_memtime();
#define PMARK(slot)                                      \
  do {                                                   \
    uint64_t t_ = __builtin_amdgcn_s_memtime();          \
    prof[slot] += t_ - pt0;                              \
    pt0 = t_;                                            \
  } while (0)
#else
#define PMARK(slot) do {} while (0)
#endif
        for (;;) {
          // re-assert uniformity of the loop-carried state (free when it already is)
          acc = (uint32_t)U((int)acc); bo = U(bo); ho = U(ho); pos = U(pos); j = U(j); mbl = U(mbl);
          insert_len = U(insert_len); copy_len = U(copy_len); dist_code = U(dist_code); distance = U(distance);
          cmd_blen = U(cmd_blen); lit_blen = U(lit_blen); dist_blen = U(dist_blen); max_dist = U(max_dist);
          dr0 = U(dr0); dr1 = U(dr1); dr2 = U(dr2); dr3 = U(dr3); dridx = U(dridx); phase = U(phase);
          c1 = U(c1); c2b = U(c2b);
          if (++guard > guard_limit) {
            HOT_SAVE();
            return MIB_E_NO_PROGRESS;
          }
          if (phase == ST_MAIN_LOOP) {   // command (:1080-1152)
            if (pos >= part_end) {   // part mode: the next part starts here
              s.running = ST_MAIN_LOOP;
              break;
            }
            if (part && pos >= U(s.pub_next)) part_publish(pos);
            if (stop_at_boundary && guard != guard0) {   // back to the fast loop
              s.running = ST_MAIN_LOOP;
              break;
            }
            if (mbl <= 0) {
              s.running = ST_BLOCK_START;
              break;
            }
            LREFILL();
            if (cmd_blen == 0) {
              HOT_SAVE();
              s.cmd_blen = decode_block_type_and_length(s, 1, s.n_cmd_types);
              s.cmd_tree_idx = s.rings[7];
              HOT_LOAD();
              cmd_tree_idx = U(s.cmd_tree_idx);
              if (tab_lds) cmd_root = U((int)t16[cmd_base + cmd_tree_idx]);
            }
            cmd_blen--;
            PMARK(8);
            LFILL16();
            const int sym = __builtin_amdgcn_readfirstlane(tab_lds ? lsym16(cmd_root) : lsym(cmd_h, cmd_tree_idx));
            const int cbits = kCmdLut[4 * sym], ins_off = kCmdLut[4 * sym + 1], copy_off = kCmdLut[4 * sym + 2];
            dist_code = kCmdLut[4 * sym + 3];
            PMARK(9);
            LFILL16();
            const int ib = cbits & 0xFF;
            insert_len = ins_off + (ib <= 16 ? lbits(ib) : lmany(ib));
            LFILL16();
            const int cb = cbits >> 8;
            copy_len = copy_off + (cb <= 16 ? lbits(cb) : lmany(cb));
            j = 0;
            phase = ST_INSERT_LOOP;
            PMARK(0);
          }
          if (phase <= ST_INSERT_LOOP) {   // literals (:1154-1276)
            int stop = 0;
            while (j < insert_len) {
              LREFILL();
              if (lit_blen == 0) {
                HOT_SAVE();
                lit_block_switch(s);
                if (!s.trivial_lit_ctx) build_ctx_tree_base(s);
                HOT_LOAD();
              }
              int a = insert_len - j, b = lit_blen, c2 = fence - pos, d = 2031 - ho;
              int batch = a < b ? a : b;
              if (c2 < batch) batch = c2;
              if (d < batch) batch = d;
              if (d <= 0 && batch <= 0 && a > 0 && b > 0 && c2 > 0) batch = 1;   // Bug J fix
              lit_blen = U(lit_blen - batch);
              const int end = U(j + batch);
              PMARK(10);
              // 16-bit LDS tables: the context's root is one lookup, (p1 << 3 | lut1[p2]),
              // and lut1 of the literal just decoded is fetched beside it for the next one
              auto lit_run16 = [&]() {
                acc = (uint32_t)U((int)acc);
                bo = U(bo);
                ho = U(ho);
                j = U(j);
                pos = U(pos);
                // literals are gathered in a VGPR (lane = position & 63, v_writelane) and
                // stored one 64-byte line at a time: one store request per line instead of
                // one per byte, so the copies' loads wait behind far fewer stores
                int fl0 = pos;
                uint32_t ob = 0;
                auto flush = [&]() {
                  const int p = (fl0 & ~63) + lane;
                  if (p >= fl0 && p < pos && p < ring_cap) ring[p] = (uint8_t)ob;
                  fl0 = pos;
                };
                if (trivial) {
                  const int root = U((int)t16[lit_tree]);
                  while (j < end) {
                    LFILL16();
                    const int val = lsym16(root);
                    ob = write_lane(ob, (uint32_t)val, (uint32_t)(pos & 63));
                    pos++;
                    j++;
                    c2b = c1;
                    c1 = val;
                    if ((pos & 63) == 0) flush();
                  }
                  c1 = U(c1);
                  c2b = U(c2b);
                } else {
                  int p1 = c1;
                  const int p2 = c2b;
                  LU8 *lut1 = clut + 256;
                  int q2 = U((int)lut1[p2]);
                  while (j < end) {
                    const int root = U((int)croot[(q2 << 8) | p1]);
                    q2 = U((int)lut1[p1]);
                    LFILL16();
                    c2b = p1;
                    p1 = U(lsym16(root));
                    ob = write_lane(ob, (uint32_t)p1, (uint32_t)(pos & 63));
                    pos++;
                    j++;
                    if ((pos & 63) == 0) flush();
                  }
                  c1 = U(p1);
                  c2b = U(c2b);
                }
                if (fl0 != pos) flush();
              };
              auto lit_run = [&](auto g) {
                if (trivial) {
                  const int root = U(g[lit_tree]);
                  while (j < end) {
                    acc = (uint32_t)U((int)acc);
                    bo = U(bo);
                    ho = U(ho);
                    LFILL16();
                    const uint32_t v = acc >> (bo & 31);
                    int off = root + (int)(v & 0xFF);
                    const int e0 = U(g[off]);
                    const int nb = e0 >> 16;
                    int val;
                    if (nb <= 8) {
                      bo += nb;
                      val = e0 & 0xFFFF;
                    } else {
                      off += e0 & 0xFFFF;
                      off += (int)((v & ((1u << nb) - 1u)) >> 8);
                      const int e1 = U(g[off]);
                      bo += (e1 >> 16) + 8;
                      val = e1 & 0xFFFF;
                    }
                    if (pos < ring_cap) ring[pos] = (uint8_t)val;   // every lane: same byte, one transaction
                    pos++;
                    j++;
                    c2b = c1;
                    c1 = val;
                  }
                  c1 = U(c1);
                  c2b = U(c2b);
                } else {
                  int p1 = c1;
                  int p2 = c2b;
                  while (j < end) {
                    const int ctx = U((int)(clut[p1] | clut[256 + p2]));
                    p2 = p1;
                    LFILL16();
                    int off = U(ctb[ctx]);
                    const uint32_t v = acc >> (bo & 31);
                    off += (int)(v & 0xFF);
                    const int e0 = U(g[off]), nb = e0 >> 16;
                    if (nb <= 8) {
                      bo += nb;
                      p1 = e0 & 0xFFFF;
                    } else {
                      off += e0 & 0xFFFF;
                      off += (int)((v & ((1u << nb) - 1u)) >> 8);
                      const int e1 = U(g[off]);
                      bo += (e1 >> 16) + 8;
                      p1 = e1 & 0xFFFF;
                    }
                    p1 = __builtin_amdgcn_readfirstlane(p1);
                    if (pos < ring_cap) ring[pos] = (uint8_t)p1;
                    pos++;
                    j++;
                  }
                  c1 = U(p1);
                  c2b = U(p2);
                }
              };
              if (tab_lds) lit_run16();
              else lit_run(lit_h);
              PMARK(11);
              wave_sync();
              if (pos >= fence) {
                s.next_running = ST_INSERT_LOOP;
                s.running = ST_INIT_WRITE;
                stop = 1;
                break;
              }
            }
            if (stop) break;
            PMARK(1);
#ifdef MIB_PROF
            prof[4] += insert_len;
#endif
            mbl -= insert_len;   // distance (:1277-1377)
            if (mbl <= 0) {
              s.running = ST_BLOCK_START;
              break;
            }
            int dc = dist_code;
            if (dc < 0) {
              distance = dr_get(dridx);
            } else {
              LREFILL();
              if (dist_blen == 0) {
                HOT_SAVE();
                s.dist_blen = decode_block_type_and_length(s, 2, s.n_dist_types);
                s.dist_ctx_map_slice = s.rings[9] << 2;
                HOT_LOAD();
                dtrees = 0;
                for (int q = 0; q < 4; q++) dtrees |= (uint32_t)s.dist_ctx_map[s.dist_ctx_map_slice + q] << (8 * q);
                dtrees = U(dtrees);
                dist_roots();
              }
              dist_blen--;
              LFILL16();
              const int dtree = (int)((dtrees >> (8 * dc)) & 0xFF);
              const uint32_t dpair = dc < 2 ? droot01 : droot23;
              dc = __builtin_amdgcn_readfirstlane(tab_lds ? lsym16((int)((dpair >> (16 * (dc & 1))) & 0xFFFF)) : lsym(dist_h, dtree));
              if (dc < 16) {
                // short codes: ring slot and value offsets (kDistIdxOff / kDistValOff, packed)
                const int idx = (dridx + (int)((0xfff0006cu >> (2 * dc)) & 3)) & 3;
                distance = dr_get(idx) + (int)((0xc298b0a626dbull >> (3 * dc)) & 7) - 3;
                if (distance < 0) {
                  HOT_SAVE();
                  return ERR(s, -12);
                }
              } else {
                // calculateDistanceLut (:705-726) in closed form
                int eb, doff;
                if (dc < 16 + ndirect) {
                  eb = 0;
                  doff = dc - 15;
                } else {
                  const int dcp = dc - ndirect - 16, hcode = dcp >> npostfix, lcode = dcp & ((1 << npostfix) - 1);
                  eb = 1 + (hcode >> 1);
                  doff = ((((2 + (hcode & 1)) << eb) - 4) << npostfix) + lcode + ndirect + 1;
                }
                int bv;
                if (bo + eb <= 32) {
                  bv = (int)((acc >> (bo & 31)) & ((1u << eb) - 1u));
                  bo += eb;
                } else {
                  LFILL16();
                  bv = eb <= 16 ? lbits(eb) : lmany(eb);
                }
                distance = doff + (bv << npostfix);
              }
            }
            if (max_dist != max_back && pos < max_back) max_dist = pos;
            else max_dist = max_back;
            if (distance > max_dist) {
              s.running = ST_USE_DICTIONARY;
              break;
            }
            if (dc > 0) {
              dridx = (dridx + 1) & 3;
              if (dridx == 0) dr0 = distance;
              else if (dridx == 1) dr1 = distance;
              else if (dridx == 2) dr2 = distance;
              else dr3 = distance;
            }
            if (copy_len > mbl) {
              HOT_SAVE();
              return ERR(s, -9);
            }
            j = 0;
            phase = ST_COPY_LOOP;
            PMARK(2);
          }
          {   // copy (:1379-1433)
            const int dist = distance, cl = copy_len - j;
            const int src = (pos - dist) & rmask;
            if (part && src < pstart) {   // the source reaches into earlier parts
              const int b = U(min(min(src + cl, pos), pstart));
              if (!part_ready_near(src, b, g_lds.part_lo[lane], g_lds.part_hi[lane], g_lds.part_seen[lane], cover_lo) &&
                  part_wait(src, b) < 0) {
                HOT_SAVE();
                return kPartFail;
              }
            }
            if (src + cl < rmask && pos + cl < rmask) {
              int lastv = 0;   // each lane's last copied byte: lanes (cl - 1) & 63, (cl - 2) & 63 end the copy
              // uniform trip counts (lane-dependent loop exits would make the whole loop nest,
              // and with it the decoder state, divergent: VGPRs instead of SGPRs)
              const int nit = U((cl + 63) >> 6);
              if (dist >= cl) {
                for (int it = 0; it < nit; it++) {
                  const int k = it * 64 + lane;
                  if (k < cl) {
                    lastv = ring[src + k];
                    ring[pos + k] = (uint8_t)lastv;
                  }
                }
              } else {
                int q = lane % dist;
                const int qstep = 64 % dist;
                for (int it = 0; it < nit; it++) {
                  const int k = it * 64 + lane;
                  if (k < cl) {
                    lastv = ring[src + q];
                    ring[pos + k] = (uint8_t)lastv;
                  }
                  q += qstep;
                  if (q >= dist) q -= dist;
                }
              }
              PMARK(12);
              if (cl >= 2) {
                c1 = __builtin_amdgcn_readlane(lastv, (cl - 1) & 63);
                c2b = __builtin_amdgcn_readlane(lastv, (cl - 2) & 63);
              } else if (cl == 1) {
                c2b = c1;
                c1 = __builtin_amdgcn_readlane(lastv, 0);
              }
              PMARK(13);
              wave_sync();
              j = copy_len;
              mbl -= cl;
              pos += cl;
            } else {
              // ring wrap and/or fence inside the copy: chunks that never read their own writes
              int cut = 0;
              while (j < copy_len) {
                const int rem = copy_len - j;
                const int room = fence - pos;
                int chunk = rem < 4096 ? rem : 4096;
                if (dist >= ring_size - 4096) chunk = rem < 64 ? rem : 64;
                if (dist >= ring_size - 64) chunk = 1;
                if (room < chunk) chunk = room;
                if (chunk < 1) chunk = 1;
                // byte p copies the byte dist back, or (overlap) its periodic image before pos
                const int base = pos - dist;
                const int nit = U((chunk + 63) >> 6);
                for (int it = 0; it < nit; it++) {
                  const int k = it * 64 + lane;
                  if (k < chunk) {
                    const int p = pos + k;
                    const int srcp = base + (dist > k ? k : k % dist);
                    const uint8_t v = ring[srcp & rmask];
                    if (p < ring_cap) ring[p] = v;
                  }
                }
                wave_sync();
                mbl -= chunk;
                pos += chunk;
                j += chunk;
                if (pos >= fence) {
                  s.next_running = ST_COPY_LOOP;
                  s.running = ST_INIT_WRITE;
                  break;
                }
              }
              if (j < copy_len) cut = 1;
              if (cut) break;
              wave_sync();
              c1 = __builtin_amdgcn_readfirstlane(ctx_byte(s, pos - 1, rmask));
              c2b = __builtin_amdgcn_readfirstlane(ctx_byte(s, pos - 2, rmask));
            }
            phase = ST_MAIN_LOOP;
            PMARK(3);
#ifdef MIB_PROF
            prof[5]++;
#endif
          }
        }
#ifdef MIB_PROF
        if (lane == 0)
          for (int q = 0; q < 16; q++) atomicAdd(&g_prof[q], (unsigned long long)prof[q]);
#endif
#undef PMARK
        HOT_SAVE();
        s.cmd_tree_idx = cmd_tree_idx;
#undef HOT_LOAD
#undef HOT_SAVE
#undef LHALF
#undef LFILL16
#undef LREFILL
#undef U
        return 0;
}


// The common case of the command loop, with no state-machine exits in it: LDS prefix
// codes, no block switch, no input refill, no ring wrap or flush, no dictionary word.
// Each command is checked up front (at its start, after its lengths, before its distance)
// and whatever does not fit is left, at exactly the state the general loop would be in at
// that point, to hot_loop (which then returns here at the next command boundary).
// Bits are read in the same order as the general loop; only the refill / block-switch /
// fence checks it makes are hoisted to where they provably cannot fire.
//
// Latency structure (one wave; every step of a command depends on the one before):
//  * bit reader: the reference's (acc, bo, ho) are tracked exactly, but the bits come from a
//    64-bit buffer holding the next two half-words as well, and the half-word after those is
//    loaded one refill AHEAD -- a refill is a register shift, never an LDS round trip;
//  * context-modelled literals: while literal k's prefix code is looked up, the lanes gather
//    the whole root row of literal k + 1 (its p2 = literal k - 1 is known; ctx_root is laid
//    out [lut1[p2]][p1]), so the next root is a readlane of the decoded symbol -- one LDS
//    round trip per literal instead of two;
//  * copies of <= 64 bytes: the source load is issued (LDS-DMA into one of kCopyQ slots) and
//    the command loop goes on; a copy is completed (its stores, and the new (p1, p2)) only
//    when something needs it: context-modelled literals (their first context is the copy's
//    last two bytes), a later copy whose source may read its destination, a full queue, or
//    the exit.  A run of copies (C4: 62 % of commands have no literals) thus keeps up to
//    kCopyQ source loads in flight instead of waiting for each before the next is issued.
template <bool kTrivial, bool kPart>
__device__ __noinline__ int fast_loop(int fence_in, int rmask_in) {
#define U(x) __builtin_amdgcn_readfirstlane(x)
  DecS &s = *(DecS *)&g_dec;
  GU8 *ring = (GU8 *)s.ring;
  LU16 *win16 = (LU16 *)g_lds.win;
  LU16 *t16 = (LU16 *)s.tab_lds;
  typedef const __attribute__((address_space(3))) uint64_t LU64;
  LU64 *croot64 = (LU64 *)g_lds.ctx_root;
  LU8 *lut1 = (LU8 *)g_lds.ctx_lut + 256;
  const int lane = LANE;
  const int rmask = U(rmask_in);
  // positions stay below lim: no fence, flush or wrap inside a command
  const int lim = kPart ? U(min(min(fence_in, rmask), s.part_end)) : U(min(fence_in, rmask));
  // part mode (a build of its own): publishing, and the 64 earlier parts' ranges / acquired
  // progress (lane l)
  constexpr bool part = kPart;
  const int pstart = kPart ? U(s.part_start) : 0, cover_lo = kPart ? U(s.cover_lo) : 0;
  int pub_next = kPart ? U(s.pub_next) : 0x7FFFFFFF;
  uint64_t *const prog_me = kPart ? s.prog + U(s.pidx) : nullptr;
  int plo = 0, phi = 0, pseen = 0;
  if (part) {
    plo = g_lds.part_lo[LANE];
    phi = g_lds.part_hi[LANE];
    pseen = g_lds.part_seen[LANE];
  }
  const int npostfix = U(s.npostfix), ndirect = U(s.ndirect), max_back = U(s.max_back);
  int pos = U(s.pos), mbl = U(s.mbl);
  // Bit reader.  The reference's reader (acc, bo, ho: engine.ts:1764-1933, fill16 / readFewBits)
  // is a function of two numbers: the bit position P (bits consumed from win[0]; P = 16 ho - 32
  // + bo) and the position F of its last fill point -- a fill leaves bo = P mod 16, so then
  // ho = (F >> 4) + 2 and bo = (F & 15) + (P - F).  The loop reads its bits at P from a 64-bit
  // window W = bits [Pw, Pw + 64) (Pw a multiple of 32) with the next word N in an SGPR and the
  // one after it in flight from LDS (Nv), so a refill is a register shift every 32 bits and
  // never waits for LDS; every fill point of the general loop is the one instruction F = P.
  // (acc, bo, ho) are rebuilt at the exit only.
  const int bo_in = U(s.bo), ho_in = U(s.ho);
  // (right after an input refill acc still holds the two half-words before win[0]: the general
  // loop reads on until they are behind it)
  if (ho_in < 2) return 0;
  int P = 16 * ho_in - 32 + bo_in;
  int F = P - bo_in + (bo_in & 15);
  int Pw = P & ~31;
  typedef const __attribute__((address_space(3))) uint32_t LU32;
  LU32 *win32 = (LU32 *)g_lds.win;
  uint64_t W = (uint64_t)(uint32_t)U((int)win32[Pw >> 5]) | ((uint64_t)(uint32_t)U((int)win32[(Pw >> 5) + 1]) << 32);
  uint32_t N = (uint32_t)U((int)win32[(Pw >> 5) + 2]);
  uint32_t Nv = win32[(Pw >> 5) + 3];
  int cmd_blen = U(s.cmd_blen), lit_blen = U(s.lit_blen), dist_blen = U(s.dist_blen), max_dist = U(s.max_dist);
  int dr0 = U(s.rings[0]), dr1 = U(s.rings[1]), dr2 = U(s.rings[2]), dr3 = U(s.rings[3]), dridx = U(s.dist_rb_idx);
  int c1 = U(ctx_byte(s, pos - 1, rmask));
  int c2b = U(ctx_byte(s, pos - 2, rmask));
  const int cmd_root = U((int)t16[s.cmd_base + s.cmd_tree_idx]);
  const int lit_root = kTrivial ? U((int)t16[s.lit_tree_idx]) : 0;
  // lut1 of the literal context mode, packed: lane l holds entries l, l + 64, l + 128, l + 192
  // as its four bytes (one readlane per lookup; a select among four registers would be
  // turned into an indexed private array)
  uint32_t lutp = 0;
  if (!kTrivial)
    lutp = (uint32_t)lut1[lane] | ((uint32_t)lut1[lane + 64] << 8) | ((uint32_t)lut1[lane + 128] << 16) |
           ((uint32_t)lut1[lane + 192] << 24);
  auto lut1_of = [lutp](int v) -> int {   // v wave-uniform
    return (int)(((uint32_t)__builtin_amdgcn_readlane((int)lutp, v & 63) >> (8 * (v >> 6))) & 0xFF);
  };
  // the ring slot idx (0..3) without branches: two bit tests, three selects
  auto ring_at = [&](int idx) -> int {
    const int lo = (idx & 1) ? dr1 : dr0, hi = (idx & 1) ? dr3 : dr2;
    return (idx & 2) ? hi : lo;
  };
  uint32_t droot01, droot23;
  {
    const int db = s.dist_base, sl = s.dist_ctx_map_slice;
    const uint8_t *dm = s.dist_ctx_map;
    const int r0 = t16[db + dm[sl]], r1 = t16[db + dm[sl + 1]], r2 = t16[db + dm[sl + 2]], r3 = t16[db + dm[sl + 3]];
    droot01 = (uint32_t)U((int)((uint32_t)r0 | ((uint32_t)r1 << 16)));
    droot23 = (uint32_t)U((int)((uint32_t)r2 | ((uint32_t)r3 << 16)));
  }
  int insert_len = 0, copy_len = 0, dist_code = 0, distance = 0, j = 0, phase = ST_MAIN_LOOP;
  uint32_t ncmd = 0;
  // Copies whose source load is in flight, oldest first: destination and length (qd*, qc*),
  // qn of them; the oldest's bytes arrive in LDS slot qhead, the next ones in the slots after
  // it.  (In registers, the loop-carried move of a newly loaded value waited for the load at
  // the back edge, whatever the order of the code: hence LDS-DMA.)  Destinations ascend, and
  // in the context-modelled build no literal lies between two pending copies (literals first
  // complete every copy), so completing them in order leaves (c1, c2b) = the last two bytes.
  // The queue's entries sit in lanes 0..3 of two VGPRs (qdv: destination, qcv: length), slot
  // k in lane k, written by v_writelane at the new copy's slot; the oldest one's are also kept
  // in SGPRs (qd0, qc0) for the overlap test and its stores.  (As eight SGPRs shifted down on
  // every completion, the selects and the compiler's phi copies cost ~40 scalar instructions a
  // copy, r05 ISA listing.)
  int qn = 0, qhead = 0;
  int qdv = 0, qcv = 0, qd0 = 0, qc0 = 0;
  static_assert(kCopyQ <= 64, "the pending queue lives in lanes");
  auto ensure = [&]() {   // at least 32 bits of W at P (every read is <= 24 bits)
    if (P - Pw >= 32) {
      W = (W >> 32) | ((uint64_t)N << 32);
      Pw += 32;
      N = (uint32_t)U((int)Nv);
      Nv = win32[(Pw >> 5) + 3];
    }
  };
  auto peek32 = [&]() -> uint32_t { return (uint32_t)(W >> (P - Pw)); };
  // extra bits after a fill point (the general loop: LFILL16, then lbits, or for more than 16
  // bits lmany -- whose force16 after the first 16 bits is a fill point too)
  auto xbits = [&](int n) -> int {
    ensure();
    F = n > 16 ? P + 16 : P;
    const int v = (int)(peek32() & ((1u << n) - 1u));
    P += n;
    return v;
  };
  auto sym16 = [&](int root) -> int {   // after a fill point (F = P)
    ensure();
    const uint32_t v = peek32();
    int off = root + (int)(v & 0xFF);
    int e = U((int)t16[off]);
    if ((e >> 12) > 8) {   // a second-level table: one branch around it, a common tail
      off += (e & 0xFFF) + (int)((v & ((1u << (e >> 12)) - 1u)) >> 8);
      e = U((int)t16[off]);
      P += 8;
    }
    P += e >> 12;
    return e & 0xFFF;
  };
  auto ho_now = [&]() -> int { return (F >> 4) + 2; };   // the reference's ho
  // Completing pending copies: their bytes arrive in LDS by DMA, which the compiler does not
  // wait for.  vmcnt counts loads, stores and LDS-DMA together, in issue order, so the oldest
  // copy's DMA has landed once at most qn - 1 vector-memory operations are outstanding: the
  // qn - 1 DMAs issued after it are among the youngest (stores issued after it only make the
  // wait longer, never too short).
  auto store_oldest = [&]() {   // the oldest copy's bytes (landed) -> the ring, (p1, p2)
    const int v = (int)g_cp[qhead][lane];
    if (lane < qc0) ring[qd0 + lane] = (uint8_t)v;
    if (!kTrivial) {   // (the trivial-context build never reads the context bytes here)
      c2b = qc0 >= 2 ? __builtin_amdgcn_readlane(v, qc0 - 2) : c1;
      c1 = __builtin_amdgcn_readlane(v, qc0 - 1);
    }
    qhead = (qhead + 1) & (kCopyQ - 1);
    qn--;
    qd0 = __builtin_amdgcn_readlane(qdv, qhead);   // (the next oldest; stale when qn = 0, unused)
    qc0 = __builtin_amdgcn_readlane(qcv, qhead);
  };
  auto complete_oldest = [&]() {
    wait_vm(qn - 1);
    store_oldest();
  };
  auto finish_copy = [&]() {   // every pending copy
    if (qn) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      while (qn) store_oldest();
    }
  };
#ifdef MIB_PROF
  uint64_t fp[5] = {0, 0, 0, 0, 0};
  uint64_t ft0 = __builtin_amdgcn_s_memtime();
#define FMARK(k)                                      \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    fp[k] += t_ - ft0;                                \
    ft0 = t_;                                         \
  } while (0)
#else
#define FMARK(k) do {} while (0)
#endif
  for (;;) {
    FMARK(4);
    // ---- command boundary: a block switch or refill goes to the general loop
    if (mbl <= 0 || cmd_blen == 0 || ho_now() > 2030 - 8) break;
    if (part && pos >= pub_next) {   // every output byte below pos is stored: publish
      // (inline: a call in this loop makes the compiler park SGPRs in VGPR lanes across it,
      // part mode's commands ran 40 % slower than the serial decoder's on the same stream)
      finish_copy();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(prog_me, (uint64_t)pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pub_next = pos + (int)kPartPublish;
    }
    const int P0 = P, F0 = F;
    F = P;
    const int sym = sym16(cmd_root);
    const int cbits = kCmdLut[4 * sym], ins_off = kCmdLut[4 * sym + 1], copy_off = kCmdLut[4 * sym + 2];
    dist_code = kCmdLut[4 * sym + 3];
    insert_len = ins_off + xbits(cbits & 0xFF);
    copy_len = copy_off + xbits(cbits >> 8);
    // literals and copy must stay inside this block type, the window and the ring
    // (32-bit: pos < 2^30 and each length < 2^24 + 2^15, so the sum cannot overflow; a 64-bit
    // compare is a VALU op on VGPRs here, and the compiler drained vmcnt before it -- every
    // command then waited for the previous command's copy load and stores)
    if (insert_len > lit_blen || pos + insert_len + copy_len >= lim ||
        ho_now() + ((insert_len * 15) >> 4) > 2030 - 12) {
      // hand the command over undecoded
      P = P0;
      F = F0;
      break;
    }
    cmd_blen--;
    FMARK(0);
    // ---- literals
    if (insert_len) {
      if (!kTrivial) finish_copy();   // (p1, p2) of the first literal
      int fl0 = pos;
      uint32_t ob = 0;
      const int end = pos + insert_len;
      // literals are gathered one per lane (lane pos & 63) and stored a
      // 64-byte line at a time; the inner loops run to the next line end, so the line check
      // is not paid per literal
      if (kTrivial && kSpecLit) {
        // One code for every literal: the entries of 64 literals-to-be are read at once, lane l
        // decoding as if a literal started at bit Pb + l (one LDS read; the second-level tables
        // per lane), and the run walks them: literal k starts at offset o, its entry is lane
        // o's (a v_readlane), the next starts at o + its length.  ~12 scalar instructions a
        // literal instead of an LDS round trip each; a new set of entries when o passes 63.
        // (kTrivial never reads the context bytes c1 / c2b: not tracked here.)
        int Pb = P, o = 0, last = P;
        bool fresh = true;
        int ent = 0;
        while (pos < end) {
          const int seg_end = U(min(end, (pos | 63) + 1));
          while (pos < seg_end) {
            if (fresh || o >= 64) {
              Pb += o;
              o = 0;
              fresh = false;
              // the 128 bits from Pw = Pb & ~31 (the handover test keeps them inside win)
              const int pw = Pb & ~31;
              const uint32_t w0 = win32[pw >> 5], w1 = win32[(pw >> 5) + 1], w2 = win32[(pw >> 5) + 2],
                             w3 = win32[(pw >> 5) + 3];
              const uint32_t ol = (uint32_t)(Pb - pw) + (uint32_t)lane;   // < 95
              const uint32_t lo = ol < 32 ? w0 : ol < 64 ? w1 : w2, hi = ol < 32 ? w1 : ol < 64 ? w2 : w3;
              const uint32_t bits = __builtin_amdgcn_alignbit(hi, lo, ol);   // 32 bits at Pb + lane
              const int i1 = lit_root + (int)(bits & 0xFF);
              ent = t16[i1];
              if (ent >= 0x9000)   // a second-level table (per lane); its length + the 8 root bits
                ent = t16[i1 + (ent & 0xFFF) + (int)((bits & ((1u << (ent >> 12)) - 1u)) >> 8)] + (8 << 12);
            }
            const int ek = __builtin_amdgcn_readlane(ent, o);
            last = Pb + o;
            ob = write_lane(ob, (uint32_t)(ek & 0xFFF), (uint32_t)(pos & 63));
            o += ek >> 12;
            pos++;
          }
          if ((pos & 63) == 0) {
            const int p = (fl0 & ~63) + lane;
            if (p >= fl0) ring[p] = (uint8_t)ob;
            fl0 = pos;
          }
        }
        // the reader after the run: position, fill point (the last literal's start), window
        P = Pb + o;
        F = last;
        Pw = P & ~31;
        W = (uint64_t)(uint32_t)U((int)win32[Pw >> 5]) | ((uint64_t)(uint32_t)U((int)win32[(Pw >> 5) + 1]) << 32);
        N = (uint32_t)U((int)win32[(Pw >> 5) + 2]);
        Nv = win32[(Pw >> 5) + 3];
      } else if (kTrivial && kVlit) {
        // one code: entry (LDS) -> its length -> the next entry, the chain in VGPRs (as below)
        ensure();
        uint32_t vlo = (uint32_t)W, vhi = (uint32_t)(W >> 32), vn = N, vnv = Nv;
        int vP = P, vPw = Pw, vF = F;
        int vc1 = c1, vc2 = c2b;
        while (pos < end) {
          const int seg_end = U(min(end, (pos | 63) + 1));
          while (pos < seg_end) {
            const uint32_t bits = __builtin_amdgcn_alignbit(vhi, vlo, (uint32_t)(vP - vPw));
            int off = lit_root + (int)(bits & 0xFF);
            int e = t16[off];
            int sym = e & 0xFFF, len = e >> 12;
            if (__builtin_expect(U(e) >= 0x9000, 0)) {
              off += sym + (int)((bits & ((1u << len) - 1u)) >> 8);
              e = t16[off];
              sym = e & 0xFFF;
              len = 8 + (e >> 12);
            }
            vF = vP;
            vP += len;
            ob = lane == (pos & 63) ? (uint32_t)sym : ob;
            vc2 = vc1;
            vc1 = sym;
            const bool adv = vP - vPw >= 32;
            vlo = adv ? vhi : vlo;
            vhi = adv ? vn : vhi;
            vn = adv ? vnv : vn;
            vPw = adv ? vPw + 32 : vPw;
            vnv = win32[(vPw >> 5) + 3];
            pos++;
          }
          if ((pos & 63) == 0) {
            const int p = (fl0 & ~63) + lane;
            if (p >= fl0) ring[p] = (uint8_t)ob;
            fl0 = pos;
          }
        }
        P = U(vP);
        F = U(vF);
        Pw = U(vPw);
        W = (uint64_t)(uint32_t)U((int)vlo) | ((uint64_t)(uint32_t)U((int)vhi) << 32);
        N = (uint32_t)U((int)vn);
        Nv = vnv;
        c1 = U(vc1);
        c2b = U(vc2);
      } else if (kTrivial) {
        while (pos < end) {
          const int seg_end = U(min(end, (pos | 63) + 1));
          while (pos < seg_end) {
            F = P;
            const int val = sym16(lit_root);
            ob = write_lane(ob, (uint32_t)val, (uint32_t)(pos & 63));
            pos++;
            c2b = c1;
            c1 = val;
          }
          if ((pos & 63) == 0) {
            const int p = (fl0 & ~63) + lane;
            if (p >= fl0) ring[p] = (uint8_t)ob;
            fl0 = pos;
          }
        }
      } else if (kVlit) {
        // The chain in VGPRs (every lane holds the same values): table entry (LDS) -> symbol ->
        // the next literal's root, ctx_root[lut1[p2] << 8 | p1] (LDS) -> the next entry.  Two
        // LDS round trips and a few VALU ops per literal; the bits at P come from the 64-bit
        // window W while the root read is in flight.  (The scalar form -- readfirstlane of the
        // entry, the root from a gathered row by v_readlane -- took ~450 cycles a literal: an LDS
        // read crossing to SGPRs costs ~120 cycles and a dependent v_readlane ~80, against ~70
        // for an LDS read feeding VALU ops, scripts/probe/chain_probe.hip on the MI355X.)
        // The bits come from a 128-bit window w0..w3 at pw (a multiple of 32) with the offset
        // of P in it below 64, in a VGPR for the extraction and in an SGPR for the refill test
        // (taken every ~10 literals: the window moves by 64 bits).
        ensure();   // P - Pw < 32
        LU8 *lut1b = (LU8 *)g_lds.ctx_lut + 256;
        LU16 *croot = (LU16 *)g_lds.ctx_root;
        uint32_t w0 = (uint32_t)W, w1 = (uint32_t)(W >> 32), w2 = N, w3 = Nv;
        int pw = Pw, so = P - Pw;
        uint32_t vo = (uint32_t)so;
        int vF = F;
        int vc1 = c1, vc2 = c2b;
        int vroot = croot[(lut1b[c2b] << 8) | c1];
        uint32_t vcls = lut1b[c1];   // lut1[p2] of the next literal
        while (pos < end) {
          const int seg_end = U(min(end, (pos | 63) + 1));
          while (pos < seg_end) {
            const bool up = vo >= 32u;
            const uint32_t bits = __builtin_amdgcn_alignbit(up ? w2 : w1, up ? w1 : w0, vo);   // 32 bits at P
            // (LDS byte addresses as index * 2 + a base ready early: one v_lshl_add on the chain)
            const uint32_t tb = lds_addr(t16) + ((bits & 0xFF) << 1);
            const uint32_t ea = lshl1_add((uint32_t)vroot, tb);
            int e = *(LU16 *)(uintptr_t)ea;
            int sym = e & 0xFFF, len = e >> 12;
            const uint32_t cb = lds_addr(croot) + (vcls << 9);
            // the next root and context class, issued before the second-level test resolves
            int nroot = *(LU16 *)(uintptr_t)lshl1_add((uint32_t)sym, cb);
            uint32_t ncls = lut1b[sym];
            const int se = U(e);
            int slen = se >> 12;
            if (__builtin_expect(se >= 0x9000, 0)) {   // a second-level table (uniform branch)
              // (the first reads are used on this path too, so they are not sunk below the
              // branch; the results replace them in place, so the common path copies nothing)
              asm volatile("; %0 %1" ::"v"(nroot), "v"(ncls));
              const int e2 = *(LU16 *)(uintptr_t)(ea + 2u * (sym + ((bits & ((1u << len) - 1u)) >> 8)));
              const int sym2 = e2 & 0xFFF, len2 = 8 + (e2 >> 12);
              const int nroot2 = *(LU16 *)(uintptr_t)lshl1_add((uint32_t)sym2, cb);
              const uint32_t ncls2 = lut1b[sym2];
              asm volatile("v_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\tv_mov_b32 %2, %6\n\tv_mov_b32 %3, %7"
                           : "+v"(nroot), "+v"(ncls), "+v"(sym), "+v"(len)
                           : "v"(nroot2), "v"(ncls2), "v"(sym2), "v"(len2));
              slen = U(len2);
            }
            vF = pw + (int)vo;
            vo += (uint32_t)len;
            so += slen;
            ob = lane == (pos & 63) ? (uint32_t)sym : ob;
            vc2 = vc1;
            vc1 = sym;
            vroot = nroot;
            vcls = ncls;
            if (so >= 64) {   // the window moves by 64 bits (a literal takes <= 15)
              pw += 64;
              so -= 64;
              vo -= 64u;
              w0 = w2;
              w1 = w3;
              w2 = win32[(pw >> 5) + 2];
              w3 = win32[(pw >> 5) + 3];
            }
            pos++;
          }
          if ((pos & 63) == 0) {
            const int p = (fl0 & ~63) + lane;
            if (p >= fl0) ring[p] = (uint8_t)ob;
            fl0 = pos;
          }
        }
        // back to the scalar state (the reader's window reloaded at P)
        P = pw + so;
        F = U(vF);
        Pw = P & ~31;
        W = (uint64_t)(uint32_t)U((int)win32[Pw >> 5]) | ((uint64_t)(uint32_t)U((int)win32[(Pw >> 5) + 1]) << 32);
        N = (uint32_t)U((int)win32[(Pw >> 5) + 2]);
        Nv = win32[(Pw >> 5) + 3];
        c1 = U(vc1);
        c2b = U(vc2);
      } else {
        int root = U((int)g_lds.ctx_root[(lut1_of(c2b) << 8) | c1]);
        while (pos < end) {
          const int seg_end = U(min(end, (pos | 63) + 1));
          while (pos < seg_end) {
            // the root row of the next literal (its p2 is the current c1), 4 entries per lane
            const uint64_t row = croot64[(lut1_of(c1) << 6) | lane];
            F = P;
            c2b = c1;
            c1 = U(sym16(root));
            const uint64_t e = c1 & 2 ? row >> 32 : row;   // lane c1 >> 2 holds entries 4 (c1 >> 2) ..
            root = __builtin_amdgcn_readlane((int)(uint32_t)(e >> (16 * (c1 & 1))), c1 >> 2) & 0xFFFF;
            ob = write_lane(ob, (uint32_t)c1, (uint32_t)(pos & 63));
            pos++;
          }
          if ((pos & 63) == 0) {
            const int p = (fl0 & ~63) + lane;
            if (p >= fl0) ring[p] = (uint8_t)ob;
            fl0 = pos;
          }
        }
      }
      if (fl0 != pos) {
        const int p = (fl0 & ~63) + lane;
        if (p >= fl0 && p < pos) ring[p] = (uint8_t)ob;
      }
      lit_blen -= insert_len;
    }
    ncmd++;
    FMARK(1);
    // ---- distance: anything unusual hands over with the literals done
    j = insert_len;
    phase = ST_INSERT_LOOP;
    if (mbl - insert_len <= 0 || (dist_code >= 0 && dist_blen == 0) || ho_now() > 2030 - 8) break;
    const int dP = P, dF = F, dmax = max_dist;
    int dc = dist_code;
    if (dc < 0) {
      distance = ring_at(dridx);
    } else {
      F = P;
      const uint32_t dpair = dc < 2 ? droot01 : droot23;
      dc = U(sym16((int)((dpair >> (16 * (dc & 1))) & 0xFFFF)));
      if (dc < 16) {
        const int idx = (dridx + (int)((0xfff0006cu >> (2 * dc)) & 3)) & 3;
        distance = ring_at(idx) + (int)((0xc298b0a626dbull >> (3 * dc)) & 7) - 3;
      } else {
        int eb, doff;
        if (dc < 16 + ndirect) {
          eb = 0;
          doff = dc - 15;
        } else {
          const int dcp = dc - ndirect - 16, hcode = dcp >> npostfix, lcode = dcp & ((1 << npostfix) - 1);
          eb = 1 + (hcode >> 1);
          doff = ((((2 + (hcode & 1)) << eb) - 4) << npostfix) + lcode + ndirect + 1;
        }
        // (the general loop: lbits while they fit its 32-bit accumulator, else a fill first)
        int bv;
        if ((F & 15) + (P - F) + eb <= 32) {
          ensure();
          bv = (int)(peek32() & ((1u << eb) - 1u));
          P += eb;
        } else {
          bv = xbits(eb);
        }
        distance = doff + (bv << npostfix);
      }
    }
    if (max_dist != max_back && pos < max_back) max_dist = pos;
    else max_dist = max_back;
    const int src = (pos - distance) & rmask;
    if (distance < 0 || distance > max_dist || copy_len > mbl - insert_len || src + copy_len >= rmask) {
      // error, dictionary word or wrapping copy: redo the distance in the general loop
      P = dP;
      F = dF;
      max_dist = dmax;
      break;
    }
    if (part && src < pstart) {   // the source reaches into earlier parts: wait until they wrote it
      const int b = U(min(min(src + copy_len, pos), pstart));
      if (!part_ready_near(src, b, plo, phi, pseen, cover_lo)) {
        // not yet known to be written: the general loop redoes the distance and waits (no
        // call in this loop, above)
        P = dP;
        F = dF;
        max_dist = dmax;
        break;
      }
    }
    mbl -= insert_len;
    if (dist_code >= 0) dist_blen--;
    if (dc > 0) {
      dridx = (dridx + 1) & 3;
      dr0 = dridx == 0 ? distance : dr0;   // (selects: the if-chain compiled to branches)
      dr1 = dridx == 1 ? distance : dr1;
      dr2 = dridx == 2 ? distance : dr2;
      dr3 = dridx == 3 ? distance : dr3;
    }
    FMARK(2);
    // ---- copy (no wrap, no fence)
    {
      const int cl = copy_len, dist = distance;
      // Every copy load below is unconditional (lanes past the copy read an in-range byte):
      // a load under an exec-masked branch can stay outstanding on the path that skips the
      // branch, and the compiler then drains vmcnt at an unrelated later reuse of its
      // register -- it did so inside the literal loop, once per literal.
      if (cl <= 64) {   // one lane per byte: issue the load, complete later
        const int q = dist >= cl ? lane : lane % dist;
        // Pending copies whose destination the source may read are completed first (the
        // destinations ascend: while the oldest starts below the source's end); then, with the
        // queue full, the oldest.  Sources far back (C4: half the distances exceed 64 KiB)
        // need neither, so the loads of a run of copies overlap.
        while (qn && src + cl > qd0) complete_oldest();
        if (qn == kCopyQ) complete_oldest();
        const int at = src + (lane < cl ? q : 0);
        typedef __attribute__((address_space(3))) void LV;
        typedef __attribute__((address_space(1))) void GV;
        const int slot = (qhead + qn) & (kCopyQ - 1);
        __builtin_amdgcn_global_load_lds((GV *)(ring + at), (LV *)g_cp[slot], 1, 0, 0);   // lane l -> dword l
        qdv = (int)write_lane((uint32_t)qdv, (uint32_t)pos, (uint32_t)slot);
        qcv = (int)write_lane((uint32_t)qcv, (uint32_t)cl, (uint32_t)slot);
        qd0 = qn == 0 ? pos : qd0;
        qc0 = qn == 0 ? cl : qc0;
        qn++;
      } else {
        finish_copy();   // (this copy may read it)
        int lastv = 0;
        const int nit = U((cl + 63) >> 6);
        const int last = cl - 1;
        if (dist >= cl && nit <= 4) {
          // up to 256 bytes: every load issued before the first store (one round trip, not nit)
          const int v0 = ring[src + min(lane, last)];
          const int v1 = ring[src + min(lane + 64, last)];
          const int v2 = ring[src + min(lane + 128, last)];
          const int v3 = ring[src + min(lane + 192, last)];
          if (lane < cl) ring[pos + lane] = (uint8_t)v0;
          if (lane + 64 < cl) ring[pos + 64 + lane] = (uint8_t)v1;
          if (lane + 128 < cl) ring[pos + 128 + lane] = (uint8_t)v2;
          if (lane + 192 < cl) ring[pos + 192 + lane] = (uint8_t)v3;
          lastv = lane + 192 < cl ? v3 : lane + 128 < cl ? v2 : lane + 64 < cl ? v1 : v0;
        } else if (dist >= cl) {
          for (int it = 0; it < nit; it++) {
            const int k = it * 64 + lane;
            const int v = ring[src + min(k, last)];
            if (k < cl) {
              lastv = v;
              ring[pos + k] = (uint8_t)v;
            }
          }
        } else {
          int q = lane % dist;
          const int qstep = 64 % dist;
          for (int it = 0; it < nit; it++) {
            const int k = it * 64 + lane;
            const int v = ring[src + q];   // (q < dist: inside the source)
            if (k < cl) {
              lastv = v;
              ring[pos + k] = (uint8_t)v;
            }
            q += qstep;
            if (q >= dist) q -= dist;
          }
        }
        c2b = __builtin_amdgcn_readlane(lastv, (cl - 2) & 63);
        c1 = __builtin_amdgcn_readlane(lastv, (cl - 1) & 63);
      }
      mbl -= cl;
      pos += cl;
    }
    phase = ST_MAIN_LOOP;
    j = 0;
    FMARK(3);
  }
  finish_copy();
  wave_sync();
  {
    const int ho = ho_now();
    s.acc = (uint32_t)win16[ho - 2] | ((uint32_t)win16[ho - 1] << 16);
    s.bo = (F & 15) + (P - F);
    s.ho = ho;
  }
  s.pos = pos; s.mbl = mbl;
  s.cmd_blen = cmd_blen; s.lit_blen = lit_blen; s.dist_blen = dist_blen; s.max_dist = max_dist;
  s.rings[0] = dr0; s.rings[1] = dr1; s.rings[2] = dr2; s.rings[3] = dr3; s.dist_rb_idx = dridx;
  s.insert_len = insert_len; s.copy_len = copy_len; s.dist_code = dist_code; s.j = j;
  s.guard += 3ull * ncmd;
  s.running = phase;
  if (kPart) s.pub_next = pub_next;
#ifdef MIB_PROF
  if (lane == 0) {
    atomicAdd(&g_prof[14], (unsigned long long)ncmd);
    atomicAdd(&g_prof[15], 1ull);
    for (int q = 0; q < 5; q++) atomicAdd(&g_prof[8 + q], (unsigned long long)fp[q]);
  }
#endif
  return 0;
#undef U
#undef FMARK
}

// one invocation of decompress(); returns 0, 1 (done), 2 (output full / compound return) or < 0
__device__ __forceinline__ int decompress(DecS &s, int8_t *dist_extra, int32_t *dist_offset, int32_t *ctxmap_table) {
  int r;
  if (s.running < 0) return ERR(s, -28);
  if (s.running == ST_INITED) {
    fill16(s);
    int wb;
    if (bits(s, 1) == 0) wb = 16;
    else {
      int n = bits(s, 3);
      if (n) wb = 17 + n;
      else {
        n = bits(s, 3);
        if (n == 1) wb = -1;
        else if (n) wb = 8 + n;
        else wb = 17;
      }
    }
    if (wb == -1) return ERR(s, -11);
    s.max_ring = 1 << wb;
    s.max_back = s.max_ring - 16;
    s.running = ST_BLOCK_START;
  }
  int fence = s.ring_size;
  int rmask = s.ring_size - 1;
  while (s.running != ST_FINISHED) {
    if (++s.guard > s.guard_limit) return MIB_E_NO_PROGRESS;
    switch (s.running) {
      case ST_BLOCK_START:
        if (s.pos >= s.part_end) return 3;   // part mode: the next part starts here
        if (s.mbl < 0) return ERR(s, -10);
        if ((r = read_next_mb_header(s)) < 0) return r;
        fence = s.ring_size;
        if (s.pos + s.mbl <= s.ring_size) fence = 0x7FFFFFFF;
        rmask = s.ring_size - 1;
        continue;
      case ST_COMPRESSED_BLOCK_START:
        if ((r = read_codes_and_maps(s, dist_extra, dist_offset, ctxmap_table)) < 0) return r;
        s.running = ST_MAIN_LOOP;
        continue;
      case ST_MAIN_LOOP:
      case ST_INSERT_LOOP:
      case ST_COPY_LOOP: {
        if (s.running == ST_MAIN_LOOP && s.pos >= s.part_end) return 3;
        {
          int rr;
          if (s.tab16) {
            if (s.running == ST_MAIN_LOOP) {
              if (s.part) rr = s.trivial_lit_ctx ? fast_loop<true, true>(fence, rmask) : fast_loop<false, true>(fence, rmask);
              else rr = s.trivial_lit_ctx ? fast_loop<true, false>(fence, rmask) : fast_loop<false, false>(fence, rmask);
              if (rr < 0) return rr;
            }
            // what the fast loop left (a block switch, a refill, a dictionary word, a wrap,
            // the block end ...): one command of the general loop
            rr = hot_loop<true>(fence, rmask, 1);
          } else {
            rr = hot_loop<false>(fence, rmask, 0);
          }
          if (rr < 0) return rr;
        }
        if (s.part && s.pos >= s.pub_next) part_publish(s.pos);
        continue;
      }
      case ST_USE_DICTIONARY:
        if ((r = use_dictionary(s, fence)) < 0) return r;
        continue;
      case ST_COPY_FROM_COMPOUND: {
        int n = copy_from_compound(s, fence);
        if (n < 0) return n;
        s.pos += n;
        if (s.pos >= fence) {
          s.next_running = ST_COPY_FROM_COMPOUND;
          s.running = ST_INIT_WRITE;
          return 2;
        }
        s.running = ST_MAIN_LOOP;
        continue;
      }
      case ST_READ_METADATA:
        while (s.mbl > 0) {
          MAYBE_REFILL(s);
          fill16(s);
          bits(s, 8);
          s.mbl--;
        }
        s.running = ST_BLOCK_START;
        continue;
      case ST_COPY_UNCOMPRESSED: {   // :838-867
        if (s.mbl <= 0) {
          if (s.bo == 32 && (r = prepare(s)) < 0) return r;
          s.running = ST_BLOCK_START;
          continue;
        }
        int chunk = s.ring_size - s.pos < s.mbl ? s.ring_size - s.pos : s.mbl;
        if ((r = copy_raw_bytes(s, s.pos, chunk)) < 0) return r;
        s.mbl -= chunk;
        s.pos += chunk;
        if (s.pos == s.ring_size) {
          s.next_running = ST_COPY_UNCOMPRESSED;
          s.running = ST_INIT_WRITE;
          continue;
        }
        if (s.bo == 32 && (r = prepare(s)) < 0) return r;
        s.running = ST_BLOCK_START;
        continue;
      }
      case ST_INIT_WRITE:
        if (s.part) {   // part mode decodes into the output itself: nothing to flush
          s.running = s.next_running;
          continue;
        }
        s.rb_ready = s.pos < s.ring_size ? s.pos : s.ring_size;
        s.running = ST_WRITE;
        continue;
      case ST_WRITE:
        if ((r = write_ring(s)) != 0) return r;
        if (s.pos >= s.max_back) s.max_dist = s.max_back;
        if (s.pos >= s.ring_size) {
          if (s.direct && (s.next_running != ST_FINISHED || s.pos > s.ring_size)) leave_direct(s);
          if (s.pos > s.ring_size) {
            int extra = s.pos - s.ring_size;
            uint8_t v = 0;
            if (LANE < extra) v = s.ring[s.ring_size + LANE];
            wave_sync();
            if (LANE < extra) s.ring[LANE] = v;   // slack <= 37 + 64 bytes
            if (extra > 64) {
              for (int k = 64; k < extra; k++) {
                if (LANE == 0) s.ring[k] = s.ring[s.ring_size + k];
              }
            }
            wave_sync();
          }
          s.pos &= rmask;
          s.rb_written = 0;
        }
        s.running = s.next_running;
        continue;
      default:
        return ERR(s, -28);
    }
  }
  if (s.mbl < 0) return ERR(s, -10);
  if ((r = jump_to_byte_boundary(s)) != 0) return r;
  if ((r = check_health(s, 1)) != 0) return r;
  return 1;
}

// A fresh decoder state for one job (initState, engine.ts:160-178), in LDS.
__device__ void dec_init(DecS &s, const DecJob &job, uint8_t *ring, int32_t *tables, uint8_t *ctx, int32_t *block_trees,
                         uint16_t *tab, int tab_cap) {
  const int lane = LANE;
    s.l = &g_lds;
  s.in = job.in;
  s.in_len = job.in_len;
  s.in_off = 0;
  s.acc = 0;
  s.bo = 32;
  s.ho = 2048;
  s.tail = 0;
  s.eos = 0;
  s.running = 0;
  s.next_running = 0;
  s.ring = ring;
  s.ring_cap = 0;
  s.ring_size = 0;
  s.max_ring = 0;
  s.max_back = 0;
  s.max_dist = 0;
  s.expected_total = 0;
  s.pos = 0;
  s.mbl = 0;
  s.input_end = 0;
  s.is_uncompressed = 0;
  s.is_metadata = 0;
  s.lit_blen = s.n_lit_types = s.cmd_blen = s.n_cmd_types = s.dist_blen = s.n_dist_types = 0;
  for (int i = 0; i < 10; i++) s.rings[i] = 0;
  s.rings[0] = 16; s.rings[1] = 15; s.rings[2] = 11; s.rings[3] = 4;
  s.dist_rb_idx = 3;
  s.ring_scratch = ring;
  s.direct = 0;
  s.tab_lds = tab;
  s.tab_cap = tab_cap;
  s.tab16 = s.cmd_base = s.dist_base = 0;
  s.bt = block_trees;
  s.tab_hbm = tables;
  s.lit_group = tables;
  s.cmd_group = tables;
  s.dist_group = tables;
  s.ctx_modes = ctx + 256 * 64 + 256 * 4;
  s.ctx_map = ctx;
  s.dist_ctx_map = ctx + 256 * 64;
  s.trivial_lit_ctx = s.lit_tree_idx = s.cmd_tree_idx = 0;
  s.j = s.insert_len = s.copy_len = s.dist_code = s.distance = 0;
  s.ctx_map_slice = s.dist_ctx_map_slice = s.clo1 = s.clo2 = 0;
  s.npostfix = s.ndirect = 0;
  s.out = job.out;
  s.out_cap = (int64_t)job.out_cap;
  s.out_flushed = 0;
  s.known_size = job.out_size > 0;
  s.chunk_start = 0;
  s.chunk_size = s.known_size ? job.out_size : 16384;
  s.rb_written = s.rb_ready = 0;
  s.cd = job.dict;
  s.cd_total = (int)job.dict_len;
  s.cd_br_offset = s.cd_br_length = s.cd_br_copied = s.cd_br_index = 0;
  // iteration guard: far above what any stream can need (each iteration consumes input
  // bits or produces output), low enough that a bug cannot spin a GPU forever
  s.guard = 0;
  s.guard_limit = 64ull * (job.in_len + 64) * 8 + 4ull * job.out_cap + (1ull << 26);
  // initState (:160-178): fresh zeroed byteBuffer (its stale tail is observable) and block trees
  for (int i = lane; i < (int)sizeof(g_lds.win); i += 64) g_lds.win[i] = 0;
  for (int i = lane; i <= kBlockTreesCap; i += 64) block_trees[i] = 0;
  __syncthreads();
  if (lane == 0) block_trees[0] = 7;
  __syncthreads();
  s.win_base = -4096;
  s.mb_bit = 0;
  s.mb_pos = s.mb_len = 0;
  s.part = 0;
  s.part_start = 0;
  s.part_end = 0x7FFFFFFF;
  s.pub_next = 0x7FFFFFFF;
  s.pidx = 0;
  s.cover_lo = 0;
  s.pctx = 0;
  s.prog = nullptr;
  s.ppos = nullptr;
}

// Persistent grid: block b decodes jobs b, b + grid, ...  Scratch per block:
//   [ring: ring_bytes][tables: kDecodeTableInts int32][ctx maps: kDecodeCtxBytes][dist luts]
// BIG: the one-stream-per-CU build (kLdsTabBig table entries, block-type trees in LDS)
template <bool BIG>
__global__ __launch_bounds__(64) void decode_streams_kernel(DecJob *jobs, int njobs, uint8_t *scratch,
                                                            uint64_t per_block, uint64_t ring_bytes) {
  constexpr int tab_cap = BIG ? kLdsTabBig : kLdsTab;
  __shared__ uint16_t tab[tab_cap];
  __shared__ int32_t bt_lds[BIG ? kBlockTreesCap + 1 : 1];
  uint8_t *base = scratch + (uint64_t)blockIdx.x * per_block;
  uint8_t *ring = base;
  int32_t *tables = reinterpret_cast<int32_t *>(base + ring_bytes);
  uint8_t *ctx = reinterpret_cast<uint8_t *>(tables + kDecodeTableInts);
  int8_t *dist_extra = reinterpret_cast<int8_t *>(ctx + kDecodeCtxBytes);
  int32_t *dist_offset = reinterpret_cast<int32_t *>(dist_extra + 1152);
  int32_t *ctxmap_table = dist_offset + 1152;
  // the block-type trees: after the table area when the launch gave room for them
  int32_t *block_trees = BIG ? bt_lds : ctxmap_table + 1100;
  const int lane = threadIdx.x;
  for (int jb = blockIdx.x; jb < njobs; jb += gridDim.x) {
    DecJob job = jobs[jb];
    DecS &s = *(DecS *)&g_dec;
    dec_init(s, job, ring, tables, ctx, block_trees, tab, tab_cap);
    int rc = prepare(s);
    if (rc >= 0) {
      s.running = ST_INITED;
      for (;;) {
        rc = decompress(s, dist_extra, dist_offset, ctxmap_table);
        if (rc < 0) break;
        if (s.known_size) { rc = 0; break; }
        // unknown size: the reference loops while a chunk comes back full (decode.ts / engine.ts:2223-2256)
        int64_t used = s.out_flushed - s.chunk_start;
        if (used < s.chunk_size) { rc = 0; break; }
        s.chunk_start += s.chunk_size;
        if (s.chunk_size < 4194304) s.chunk_size *= 2;
      }
    }
    if (rc >= 0 && s.known_size && s.out_flushed < job.out_size) {   // zero-padded to the known size
      for (int64_t k = s.out_flushed + lane; k < job.out_size; k += 64) s.out[k] = 0;
    }
    if (lane == 0) {
      jobs[jb].status = rc < 0 ? rc : 0;
      jobs[jb].result_len = s.known_size ? job.out_size : s.out_flushed;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- part decoding
// One part of an indexed stream: decode its metablock's header, jump to the entry, run the
// state machine to the next entry, then check that the state matches it exactly.
__device__ int part_run(DecS &s, const DecJob &job, int8_t *dist_extra, int32_t *dist_offset, int32_t *ctxmap_table) {
  const PartEntry e = *(const PartEntry *)job.part_entry;
  const bool last = job.next_entry == nullptr;
  const int lane = LANE;
  if (job.total <= 0 || job.total > (1ll << 30) || e.pos > (uint64_t)job.total) return kPartFail;
  s.part = 1;
  s.pidx = job.pidx;
  s.prog = job.prog;
  s.ppos = job.ppos;
  s.part_start = (int)e.pos;
  s.part_end = last ? 0x7FFFFFFF : (int)job.ppos[job.pidx + 1];
  s.pub_next = s.part_start + (int)kPartPublish;
  {
    const int w = job.pidx - 1 - lane;
    g_lds.part_lo[lane] = w >= 0 ? (int)job.ppos[w] : 0;
    g_lds.part_hi[lane] = w >= 0 ? (int)job.ppos[w + 1] : 0;
    g_lds.part_seen[lane] = 0;
    s.cover_lo = job.pidx >= 64 ? (int)job.ppos[job.pidx - 64] : 0;
  }
  // the output is the ring: no wrap, no flush (positions stay below total <= 2^30 <= the
  // ring size, so every `& rmask` is the identity and every fence is the end)
  int rs = 1 << job.max_ring_log;
  while (rs < job.total + 64 && rs < (1 << 30)) rs <<= 1;
  s.max_ring = 1 << job.max_ring_log;
  s.max_back = s.max_ring - 16;
  s.ring = job.out;
  s.direct = 1;
  s.ring_size = rs;
  s.ring_cap = rs + 37;
  s.expected_total = (int)job.total;
  s.known_size = 1;
  int r;
  if (e.flags & kPartAtMb) {
    if ((r = part_seek(s, (int64_t)e.bit)) < 0) return kPartFail;
    s.pos = (int)e.pos;
    s.running = ST_BLOCK_START;
  } else {
    if ((r = part_seek(s, (int64_t)e.mb_bit)) < 0) return kPartFail;
    s.pos = (int)e.mb_pos;
    if ((r = read_next_mb_header(s)) < 0 || s.running != ST_COMPRESSED_BLOCK_START) return kPartFail;
    if ((r = read_codes_and_maps(s, dist_extra, dist_offset, ctxmap_table)) < 0) return kPartFail;
    if (s.mb_pos + s.mb_len < (int)e.pos) return kPartFail;
    if ((r = part_seek(s, (int64_t)e.bit)) < 0) return kPartFail;
    s.mbl = s.mb_pos + s.mb_len - (int)e.pos;
    s.pos = (int)e.pos;
    if (e.type[0] >= s.n_lit_types || e.type[1] >= s.n_cmd_types || e.type[2] >= s.n_dist_types) return kPartFail;
    s.rings[4] = e.prev[0]; s.rings[5] = e.type[0]; s.lit_blen = (int)e.blen[0];
    s.rings[6] = e.prev[1]; s.rings[7] = e.type[1]; s.cmd_blen = (int)e.blen[1];
    s.rings[8] = e.prev[2]; s.rings[9] = e.type[2]; s.dist_blen = (int)e.blen[2];
    s.ctx_map_slice = e.type[0] << 6;
    s.lit_tree_idx = s.ctx_map[s.ctx_map_slice];
    s.clo1 = s.ctx_modes[e.type[0]] << 9;
    s.clo2 = s.clo1 + 256;
    build_ctx_tree_base(s);
    s.cmd_tree_idx = e.type[1];
    s.dist_ctx_map_slice = e.type[2] << 2;
    s.running = ST_MAIN_LOOP;
  }
  s.rings[0] = (int)e.ring[3]; s.rings[1] = (int)e.ring[2]; s.rings[2] = (int)e.ring[1]; s.rings[3] = (int)e.ring[0];
  s.dist_rb_idx = 3;
  s.max_dist = s.pos < s.max_back ? s.pos : s.max_back;
  // the literal context: the two bytes before the part, from the entry (ctx_byte); the
  // previous part's output is never written here, and it checks those bytes itself
  s.pctx = (int)e.p1 | ((int)e.p2 << 8);
#ifdef MIB_PROF
  if (lane == 0 && s.pidx_g < kPartProfMax) g_part_prof[8 * s.pidx_g + 5] = __builtin_amdgcn_s_memtime();
#endif
  r = decompress(s, dist_extra, dist_offset, ctxmap_table);
  if (last) return (r == 1 && s.pos == (int)job.total) ? 0 : kPartFail;
  if (r != 3) return kPartFail;
  const PartEntry n = *(const PartEntry *)job.next_entry;
  if (n.flags & kPartAtMb) {
    // a streaming chunk ends in a byte-aligning empty metadata block and the next one starts
    // with its own index block: step over metadata blocks up to the next part's header
    for (int guard = 0; abs_bit(s) < (int64_t)n.bit && guard < 64; guard++) {
      if (s.mbl > 0 || (r = read_next_mb_header(s)) < 0 || !s.is_metadata) return kPartFail;
      if ((r = part_seek(s, abs_bit(s) + 8 * (int64_t)s.mbl)) < 0) return kPartFail;
      s.mbl = 0;
      s.running = ST_BLOCK_START;
    }
  }
  const int idx = s.dist_rb_idx;
  bool ok = abs_bit(s) == (int64_t)n.bit && s.pos == (int)n.pos &&
            s.rings[idx & 3] == (int)n.ring[0] && s.rings[(idx - 1) & 3] == (int)n.ring[1] &&
            s.rings[(idx - 2) & 3] == (int)n.ring[2] && s.rings[(idx - 3) & 3] == (int)n.ring[3];
  if (n.flags & kPartAtMb) {
    ok = ok && s.mbl == 0;
  } else {
    ok = ok && s.running == ST_MAIN_LOOP && s.mb_bit == (int64_t)n.mb_bit && s.mb_pos == (int)n.mb_pos &&
         s.rings[5] == n.type[0] && s.rings[4] == n.prev[0] && s.lit_blen == (int)n.blen[0] &&
         s.rings[7] == n.type[1] && s.rings[6] == n.prev[1] && s.cmd_blen == (int)n.blen[1] &&
         s.rings[9] == n.type[2] && s.rings[8] == n.prev[2] && s.dist_blen == (int)n.blen[2];
  }
  if (ok) {   // the bytes this part wrote (or, for a part under 2 bytes, its own entry's)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int rmask = s.ring_size - 1;
    ok = ctx_byte(s, s.pos - 1, rmask) == n.p1 && ctx_byte(s, s.pos - 2, rmask) == n.p2;
  }
  return ok ? 0 : kPartFail;
}

// Parts are taken in order from a ticket counter, so every part a wave may wait on has
// already been taken by a running wave: a part only waits on earlier parts of its stream.
// (Chunks of consecutive parts per XCD group were measured: C2 unchanged, C5 179 -> 679 ms,
// profiles/r06/r06y3.)
__device__ __forceinline__ int next_part(unsigned *ticket, int njobs) {
  int jb = 0;
  if (LANE == 0) jb = (int)atomicAdd(ticket, 1u);
  jb = __shfl(jb, 0);
  return jb < njobs ? jb : -1;
}

template <bool BIG>
__global__ __launch_bounds__(64) void decode_parts_kernel(DecJob *jobs, int njobs, uint8_t *scratch, uint64_t per_block,
                                                          unsigned *ticket) {
  constexpr int tab_cap = BIG ? kLdsTabBig : kLdsTab;
  __shared__ uint16_t tab[tab_cap];
  __shared__ int32_t bt_lds[BIG ? kBlockTreesCap + 1 : 1];
  uint8_t *base = scratch + (uint64_t)blockIdx.x * per_block;
  int32_t *tables = reinterpret_cast<int32_t *>(base);
  uint8_t *ctx = reinterpret_cast<uint8_t *>(tables + kDecodeTableInts);
  int8_t *dist_extra = reinterpret_cast<int8_t *>(ctx + kDecodeCtxBytes);
  int32_t *dist_offset = reinterpret_cast<int32_t *>(dist_extra + 1152);
  int32_t *ctxmap_table = dist_offset + 1152;
  int32_t *block_trees = BIG ? bt_lds : ctxmap_table + 1100;
  const int lane = threadIdx.x;
  for (;;) {
    const int jb = next_part(ticket, njobs);
    if (jb < 0) break;
    const DecJob job = jobs[jb];
    DecS &s = *(DecS *)&g_dec;
#ifdef MIB_PROF
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
    dec_init(s, job, job.out, tables, ctx, block_trees, tab, tab_cap);
#ifdef MIB_PROF
    s.pidx_g = jb;
    if (lane == 0 && jb < kPartProfMax) {
      unsigned long long *q = g_part_prof + 8 * jb;
      q[0] = t_start;
      q[2] = q[3] = q[4] = 0;
      unsigned hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      q[7] = hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(hw));
      q[6] = (hw & 0xF) | ((unsigned long long)blockIdx.x << 8);
    }
#endif
    int rc = part_run(s, job, dist_extra, dist_offset, ctxmap_table);
#ifdef MIB_PROF
    if (lane == 0 && jb < kPartProfMax) g_part_prof[8 * jb + 1] = __builtin_amdgcn_s_memtime();
#endif
    if (rc == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (!job.next_entry) part_publish(0x7FFFFFFF);
      else part_publish(s.pos);
    } else {
      part_fail();
    }
    if (lane == 0) {
      jobs[jb].status = rc;
      jobs[jb].result_len = rc == 0 ? s.pos : 0;
    }
    __syncthreads();
  }
}

}  // namespace mib

// A launch with at most one stream (or part) per CU runs the build that gives each its CU's
// whole LDS; a larger one the four-per-CU build.
extern "C" hipError_t mib_decode_launch(mib::DecJob *d_jobs, int njobs, uint8_t *d_scratch, uint64_t per_block,
                                        uint64_t ring_bytes, int grid, int per_cu, hipStream_t stream) {
  if (per_cu <= 1)
    hipLaunchKernelGGL(mib::decode_streams_kernel<true>, dim3(grid), dim3(64), 0, stream, d_jobs, njobs, d_scratch, per_block,
                       ring_bytes);
  else
    hipLaunchKernelGGL(mib::decode_streams_kernel<false>, dim3(grid), dim3(64), 0, stream, d_jobs, njobs, d_scratch, per_block,
                       ring_bytes);
  return hipGetLastError();
}

extern "C" hipError_t mib_decode_parts_launch(mib::DecJob *d_jobs, int njobs, uint8_t *d_scratch, uint64_t per_block,
                                              unsigned *d_ticket, int grid, int per_cu, hipStream_t stream) {
  if (per_cu <= 1)
    hipLaunchKernelGGL(mib::decode_parts_kernel<true>, dim3(grid), dim3(64), 0, stream, d_jobs, njobs, d_scratch, per_block,
                       d_ticket);
  else
    hipLaunchKernelGGL(mib::decode_parts_kernel<false>, dim3(grid), dim3(64), 0, stream, d_jobs, njobs, d_scratch, per_block,
                       d_ticket);
  return hipGetLastError();
}

extern "C" hipError_t mib_decode_init_tables(const int16_t *host_lut) {
  return hipMemcpyToSymbol(HIP_SYMBOL(mib::kCmdLut), host_lut, sizeof(int16_t) * 704 * 4);
}

// First two bytes of each stream (window bits peek for scratch sizing) in one launch.
namespace mib {
__global__ void peek_heads_kernel(const uint8_t *in, const uint64_t *offsets, int k, uint8_t *heads) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < k; i += gridDim.x * blockDim.x) {
    uint64_t a = offsets[i], n = offsets[i + 1] - a;
    for (int q = 0; q < 16; q++) heads[16 * i + q] = (uint64_t)q < n ? in[a + q] : 0;
  }
}
}  // namespace mib

extern "C" hipError_t mib_decode_peek_heads(const uint8_t *d_in, const uint64_t *d_offsets, int k, uint8_t *d_heads,
                                            hipStream_t stream) {
  hipLaunchKernelGGL(mib::peek_heads_kernel, dim3((k + 255) / 256), dim3(256), 0, stream, d_in, d_offsets, k, d_heads);
  return hipGetLastError();
}

#ifdef MIB_PROF
extern "C" int mib_debug_read_hdr_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::g_hdr_prof), sizeof(unsigned long long) * 16);
  unsigned long long z[16] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(mib::g_hdr_prof), z, sizeof(z));
  return 0;
}
extern "C" int mib_debug_read_part_prof(unsigned long long *out, int n) {
  if (n > mib::kPartProfMax) n = mib::kPartProfMax;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::g_part_prof), sizeof(unsigned long long) * 8 * n);
}
extern "C" int mib_debug_read_prof(unsigned long long *out) {
  hipMemcpyFromSymbol(out, HIP_SYMBOL(mib::g_prof), sizeof(unsigned long long) * 16);
  unsigned long long z[16] = {0};
  hipMemcpyToSymbol(HIP_SYMBOL(mib::g_prof), z, sizeof(z));
  return 0;
}
#endif
