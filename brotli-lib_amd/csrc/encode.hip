// brotli_amd: batch Brotli (RFC 7932) encoder for gfx950 -- pipeline and host orchestration.
//
// The reference's quality-11 path (countertype/brotli-lib src/encode/encode.ts:181-281 ->
// createHqZopfliBackwardReferences backward-references-hq.ts:485-608 -> storeMetaBlock
// metablock.ts:504-761) is inherently serial per stream: an insertion-ordered binary tree
// (hash-binary-tree.ts:57-153) and a forward DP over every position.  This engine keeps the
// same algorithmic family -- hash-bucketed match finding, a cost-model shortest-path parse
// over (insert, copy, distance) commands, Huffman coding of literal / command / distance
// symbols -- restructured for the GPU (kernels in enc_match / enc_parse / enc_entropy /
// enc_emit.hip):
//
//   bucket sort              every position of every stream gets a key (the hash of 6 bytes, 4 for
//                            fonts); each stream's positions are sorted by it, stably, so each
//                            bucket is a flat chain, positions ascending (enc_sort.hip)
//   find_matches             thread per sorted entry, LDS tile of the chain: the staircase of
//                            (distance, length) matches, findAllMatches-style
//   dp                       wave per 64 KiB segment: shortest path, 64 lanes relax the
//                            copy lengths of a position at once
//   backtrack -> carry -> codes + histograms -> huffman -> sizes -> offsets -> emit -> pack
//
// Segments are independent in the parse (a copy never crosses a segment end); insert
// lengths are stitched across segments by `carry`, and the distance ring's last-distance
// slot is known at every segment start, so all entropy-coding work is segment-parallel.
// The output is one valid RFC 7932 stream per input, decodable by any decoder.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "enc_common.h"

extern "C" void mib_ctx_add_time(mib_ctx *c, const char *name, double ms);
extern "C" int mib_ctx_profiling(mib_ctx *c);
extern "C" void **mib_ctx_enc_ws(mib_ctx *c);
extern "C" void **mib_ctx_lane_ws(mib_ctx *c, int l);
extern "C" void *mib_ctx_lane_stream(mib_ctx *c, int l);
extern "C" uint8_t *mib_ctx_stage(mib_ctx *c, int slot, uint64_t need);

// ====================================================================== host orchestration
using namespace mib;
using namespace mib::enc;

extern "C" mib_ctx *mib_default_ctx(void);
extern "C" void mib_default_lock(int on);
extern "C" int mib_ctx_ready(mib_ctx *c);
extern "C" void *mib_ctx_stream_of(mib_ctx *c);
extern "C" int mib_ctx_device_of(mib_ctx *c);
extern "C" void mib_ctx_clear_times(mib_ctx *c);

namespace {

#define CK(x)                                                                                         \
  do {                                                                                                \
    hipError_t e_ = (x);                                                                              \
    if (e_ != hipSuccess) {                                                                           \
      fprintf(stderr, "brotli_amd encode: %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return MIB_E_NO_DEVICE;                                                                         \
    }                                                                                                 \
  } while (0)

struct Workspace {
  size_t cap = 0;
  uint8_t *buf = nullptr;
  uint64_t need = 0;   // the most the calls since the last trim needed (mib_encode_ws_trim's hysteresis)
  int quiet = 0;
  // a second stream for the launch pairs that do not depend on each other (the block split's
  // two state counts; the prefix codes and the metablock header): a call of few metablocks
  // runs each pair's few blocks side by side instead of back to back (cadence 291 -> 326 MB/s)
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
};

// fork: side waits for what st has queued; join: st waits for what side has queued since
struct Fork {
  hipStream_t st, side;
  hipEvent_t f, j;
  void fork() {
    if (side == st) return;
    hipEventRecord(f, st);
    hipStreamWaitEvent(side, f, 0);
  }
  void join() {
    if (side == st) return;
    hipEventRecord(j, side);
    hipStreamWaitEvent(st, j, 0);
  }
};
Fork fork_of(Workspace *ws, hipStream_t st) {
  if (!ws->side) {   // (on st's device: a workspace belongs to one context)
    int cur = -1, dev = -1;
    hipGetDevice(&cur);
    if (hipStreamGetDevice(st, &dev) == hipSuccess && dev >= 0 && dev != cur) hipSetDevice(dev);
    if (hipStreamCreateWithFlags(&ws->side, hipStreamNonBlocking) != hipSuccess) ws->side = nullptr;
    else if (hipEventCreateWithFlags(&ws->fork_ev, hipEventDisableTiming) != hipSuccess ||
             hipEventCreateWithFlags(&ws->join_ev, hipEventDisableTiming) != hipSuccess) {
      hipStreamDestroy(ws->side);
      ws->side = nullptr;
    }
    if (dev >= 0 && dev != cur) hipSetDevice(cur);
  }
  return ws->side ? Fork{st, ws->side, ws->fork_ev, ws->join_ev} : Fork{st, st, nullptr, nullptr};
}

struct Arena {
  uint8_t *base;
  size_t off = 0;
  template <class T>
  T *take(size_t n) {
    off = (off + 255) & ~(size_t)255;
    T *p = reinterpret_cast<T *>(base + off);
    off += sizeof(T) * std::max<size_t>(n, 1);
    return p;
  }
};

// candidates examined per position (the reference's tree depth / chain length by quality:
// hash-binary-tree.ts:60 maxTreeSearchDepth 64 at q11, 16 at q10; hash-chain.ts by quality)
int depth_for_quality(int q) {
  if (q >= 11) return 64;
  if (q == 10) return 32;
  if (q >= 5) return 16;
  if (q >= 2) return 4;
  return 1;
}

struct Timer {
  mib_ctx *c;
  hipStream_t s;
  bool on;
  std::vector<std::pair<const char *, std::pair<hipEvent_t, hipEvent_t>>> ev;
  void start(const char *name) {
    if (!on) return;
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a, s);
    ev.push_back({name, {a, b}});
  }
  void stop() {
    if (on) hipEventRecord(ev.back().second.second, s);
  }
  void collect() {
    for (auto &e : ev) {
      float ms = 0;
      hipEventElapsedTime(&ms, e.second.first, e.second.second);
      mib_ctx_add_time(c, e.first, ms);
      hipEventDestroy(e.second.first);
      hipEventDestroy(e.second.second);
    }
    ev.clear();
  }
};

// One stream of a call: where its bytes are and how it is framed.
struct StreamDesc {
  const uint8_t *d_data;
  uint64_t n;
  uint32_t hdr_lgwin;
  uint32_t final_;
  int32_t dc[4];
  uint32_t prev_bytes;   // p1 | p2 << 8 before data[0] (streaming)
  uint32_t hist;         // streaming: history bytes before data[0] (device-resident, contiguous)
  uint32_t abs_base;     // streaming: stream position of data[0]
  uint32_t win_abs;      // min(stream position of data[0], 2^24) (dictionary distances)
  uint32_t *hist_tab;    // streaming: the encoder's bucket table (null: none)
  uint64_t out_base;     // streaming: stream bytes emitted before this chunk
  bool streaming;        // a BrotliEncoder chunk (part index whenever it has segments to split)
  const uint8_t *cdict;  // custom dictionary (device), or null
  uint32_t cdict_len, cdict_tail4;
};

// Streams that get a part index (parts.h): one-shot streams of at least kPartMinStream bytes
// and streaming chunks, when they have more than one parse segment.  MIB_PART_MIN (bytes)
// overrides the one-shot threshold (0 disables the index).
uint64_t part_min_stream() {
  static uint64_t v = [] {
    const char *e = knob("MIB_PART_MIN");
    return e ? (uint64_t)strtoull(e, nullptr, 10) : kPartMinStream;
  }();
  return v;
}
uint32_t env_u32(const char *name, uint32_t dflt, uint32_t lo, uint32_t hi) {
  const char *e = knob(name);
  if (!e) return dflt;
  const unsigned long v = strtoul(e, nullptr, 10);
  return (uint32_t)std::max<unsigned long>(lo, std::min<unsigned long>(hi, v));
}
// part size (log2) and source lag (MIB_PART_BITS / MIB_PART_LAG override, for experiments)
uint32_t part_bits() {
  static uint32_t v = env_u32("MIB_PART_BITS", kPartBits, kSegBits, 22);
  return v;
}
uint32_t part_lag() {
  static uint32_t v = env_u32("MIB_PART_LAG", kPartLag, 0, 1u << 20);
  return v;
}
// zopfli iterations at quality 11 (MIB_ZOPFLI_ITERS overrides, for experiments)
uint32_t zopfli_iterations() {
  static uint32_t v = env_u32("MIB_ZOPFLI_ITERS", 2, 1, 2);
  return v;
}
// bytes at the start of each segment the first iteration parses when it only feeds the
// model (MIB_ZOPFLI_SAMPLE; >= 64 KiB parses whole segments)
uint32_t zopfli_sample() {
  static uint32_t v = env_u32("MIB_ZOPFLI_SAMPLE", 2048, 1024, kSeg);
  return v;
}
bool wants_parts(const StreamDesc &d) {
  const uint64_t lim = part_min_stream();
  if (lim == 0 || d.n <= kSeg) return false;
  return d.streaming || d.n >= lim;
}

struct Params {
  int quality, lgwin, npostfix, ndirect;
  bool font;
};

Params make_params(const mib_enc_opts *o) {
  Params p;
  p.quality = std::max(0, std::min(11, o ? o->quality : 11));
  p.lgwin = std::max(10, std::min(24, o ? o->lgwin : 22));
  p.npostfix = 0;
  p.ndirect = 0;
  p.font = o && o->mode == MIB_MODE_FONT;
  if (p.quality >= 4 && o && o->mode == MIB_MODE_FONT) {   // sanitizeParams (enc-constants.ts:117-127)
    p.npostfix = 1;
    p.ndirect = 12;
  }
  return p;
}

// The last-distance copies pass (rep_kernel) and 4-byte bucket keys: FONT mode, whose glyph
// records repeat with a few bytes changed (C3: -0.9 % and -1.8 % bytes; text gains < 0.01 %
// from the pass and loses from the shorter keys).  MIB_REP / MIB_HASH_BYTES override.
// Parse pieces per segment (2^shift, 8 KiB pieces): the DP is one wave per two segments and
// latency-bound, so a call with few segments runs it at low occupancy (C2's 64 MiB stream is
// 1,024 segments, one wave per SIMD), and even a full batch finishes its waves unevenly.
// Pieces cut the parse more often (a piece's first node starts a fresh path; copies stop at
// the piece end): C4 dp 123 -> 105 ms for +0.03 % bytes, C2 39 -> 8.5 ms.
// MIB_DP_PIECES=0..3 overrides.
constexpr uint64_t kSmallStream = 1ull << 20;
// Pieces per segment (2^shift) by the stream itself, so a stream parses the same in any batch:
// 8 KiB pieces; 2 KiB for one-shot streams below 1 MiB -- a lone small stream gets 512 DP waves
// per MiB instead of 128 --, 1 KiB for one-shot streams of one segment, 512 B for streaming
// chunks of up to 4 MiB (a reference-cadence
// update()'s 1 MiB chunk: its parse was 4.7 of the 9.2 ms an update took with 8 KiB pieces,
// r05m, 1.2 ms with 2 KiB, r05n; 1 KiB: 205 -> 227 MB/s for 0.38309 -> 0.38317, r05ad; 512 B:
// 330 -> 353 MB/s for 0.38326 -> 0.38341, r06 kn_pieces: two DP waves a SIMD).  C4's
// 1 MiB buffers keep 8 KiB pieces (2 KiB: 0.36296 vs 0.36281, r05n).  (MIB_DP_PIECES, experiment
// builds: one shift for every stream.)
int dp_piece_shift(uint64_t n, bool streaming) {
  static const int v = knob("MIB_DP_PIECES") ? std::min(kMaxPieceShift, std::max(0, atoi(knob("MIB_DP_PIECES")))) : -1;
  if (v >= 0) return v;
  if (streaming) return n <= 4 * kSmallStream ? 7 : 3;
  return n <= kSeg ? 6 : n < kSmallStream ? 5 : 3;   // (one segment: C1's 45,000 B, 3.65 -> 3.14 ms for +0.06 %, r05af)
}
bool rep_pass(const Params &p) {
  static const int v = knob("MIB_REP") ? atoi(knob("MIB_REP")) : -1;
  return v < 0 ? p.font : v != 0;
}
// the short scan before the tree (near_matches_kernel), at q10+ outside FONT mode: there the
// 4-byte keys already offer 4-5 byte copies and the scan's 2-3 byte ones changed C3 by -0.02 %
// for 10 % of its encode time (r05g); text's 6-byte keys offer none (C4 -0.23 %).
// (MIB_NEAR, experiment builds: 0 off, 2 every mode)
bool near_scan(const Params &p) {
  static const int v = knob("MIB_NEAR") ? atoi(knob("MIB_NEAR")) : 1;
  return p.quality >= 10 && (v == 2 || (v == 1 && !p.font));
}
// distance-cache candidates in the parse (dp_kernel KC) at q10+, every mode
// (MIB_DP_CACHE=0 turns them off: experiment builds)
int g_no_dp_cache = 0;   // mib_force_no_dp_cache (tests)
bool dp_cache(const Params &p) {
  static const int v = knob("MIB_DP_CACHE") ? atoi(knob("MIB_DP_CACHE")) : 1;
  return p.quality >= 10 && v != 0 && !__atomic_load_n(&g_no_dp_cache, __ATOMIC_RELAXED);
}
int hash_bytes(const Params &p) {
  static const int v = knob("MIB_HASH_BYTES") ? std::min(6, std::max(4, atoi(knob("MIB_HASH_BYTES")))) : -1;
  return v > 0 ? v : p.font ? 4 : kHashBytes;
}

// The static dictionary for the match finder (§8 f3), once per device: the word-list offsets
// per length and the RFC 7932 words (dict_data), and buckets of kDictWays words by their first
// four bytes, longest first (dict_tab: length << 16 | index, 0 = empty).
const uint8_t kHostDict[] = {
#include "rfc_dictionary.inc"
};
const uint8_t kHostDictSizeBits[25] = {0, 0, 0, 0, 10, 10, 11, 11, 10, 10, 10, 10, 10, 9, 9, 8, 7, 7, 8, 7, 7, 6, 6, 5, 5};
struct DictDev {
  uint8_t *data = nullptr;
  uint32_t *tab = nullptr;
};
constexpr int kDictDevices = 64;
DictDev g_dict[kDictDevices];
std::mutex g_dict_mu;
// MIB_DICT=0 turns the dictionary references off (experiments)
bool dict_enabled() {
  static bool v = [] {
    const char *e = knob("MIB_DICT");
    return !e || atoi(e) != 0;
  }();
  return v;
}
// stream positions where words are looked up (MIB_DICT_SPAN overrides): a word reference
// pays where the window has little to offer, and each one costs the decoder a trip through
// its general loop
uint32_t dict_span() {
  static uint32_t v = env_u32("MIB_DICT_SPAN", 1u << 16, 0, 1u << 30);
  return v;
}
const DictDev *dict_device(int dev) {
  if (dev < 0 || dev >= kDictDevices) return nullptr;
  std::lock_guard<std::mutex> lk(g_dict_mu);
  DictDev &d = g_dict[dev];
  if (d.data) return &d;
  std::vector<uint32_t> off(32, 0);
  for (int L = 4; L < 25; L++) off[L + 1] = off[L] + ((uint32_t)L << kHostDictSizeBits[L]);
  for (int L = 26; L < 32; L++) off[L] = off[25];
  std::vector<uint8_t> blob(128 + sizeof(kHostDict));
  memcpy(blob.data(), off.data(), 128);
  memcpy(blob.data() + 128, kHostDict, sizeof(kHostDict));
  std::vector<uint32_t> tab((size_t)kDictWays << kDictHashBits, 0u);
  for (int L = 24; L >= 4; L--)
    for (uint32_t i = 0; i < (1u << kHostDictSizeBits[L]); i++) {
      const uint8_t *w = kHostDict + off[L] + i * L;
      const uint32_t w4 = (uint32_t)w[0] | ((uint32_t)w[1] << 8) | ((uint32_t)w[2] << 16) | ((uint32_t)w[3] << 24);
      uint32_t *slot = tab.data() + (size_t)((w4 * 0x1E35A7BDu) >> (32 - kDictHashBits)) * kDictWays;
      for (int k = 0; k < kDictWays; k++)
        if (!slot[k]) {
          slot[k] = ((uint32_t)L << 16) | i;
          break;
        }
    }
  uint8_t *dd = nullptr;
  uint32_t *dt = nullptr;
  if (hipMalloc(&dd, blob.size()) != hipSuccess) return nullptr;
  if (hipMalloc(&dt, tab.size() * 4) != hipSuccess) {
    hipFree(dd);
    return nullptr;
  }
  if (hipMemcpy(dd, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dt, tab.data(), tab.size() * 4, hipMemcpyHostToDevice) != hipSuccess) {
    hipFree(dd);
    hipFree(dt);
    return nullptr;
  }
  d.data = dd;
  d.tab = dt;
  return &d;
}

// Encode a group of streams into d_out (packed from out_pos; returns the per-stream sizes).
int encode_group(mib_ctx *ctx, const Params &prm, const StreamDesc *sd, size_t k, uint8_t *d_out, uint64_t out_cap,
                 uint64_t out_pos, uint64_t *sizes, int32_t (*dc_out)[4], hipStream_t st, void **ws_slot) {
  std::vector<Job> jobs(k);
  std::vector<Seg> segs;
  std::vector<Mb> mbs;
  std::vector<uint32_t> seg_job;   // per 64 KiB of global positions: its stream
  std::vector<SegRef> seg_ref;     // ... and where its bytes are
  uint64_t pos_total = 0, out_scratch = 0, cmd_total = 0, npieces = 0;
  bool any_hist = false, any_parts = false, any_dict = false, any_cdict = false;
  for (size_t j = 0; j < k; j++) {
    Job &jb = jobs[j];
    memset(&jb, 0, sizeof(jb));
    const uint64_t n = sd[j].n;
    jb.data = sd[j].d_data;
    jb.n = (uint32_t)n;
    jb.lgwin = (uint32_t)prm.lgwin;
    jb.npostfix = (uint32_t)prm.npostfix;
    jb.ndirect = (uint32_t)prm.ndirect;
    jb.uncompressed = (prm.quality == 0 || n < 64) ? 1 : 0;
    jb.font = prm.font ? 1 : 0;
    jb.hq = prm.quality >= 10 ? 1 : 0;
    jb.hdr_lgwin = sd[j].hdr_lgwin;
    jb.final_ = sd[j].final_;
    for (int q = 0; q < 4; q++) jb.dc_in[q] = jb.dc_out[q] = sd[j].dc[q];
    jb.prev_bytes = sd[j].prev_bytes;
    jb.hist = sd[j].hist;
    jb.abs_base = sd[j].abs_base;
    jb.win_abs = sd[j].win_abs;
    jb.hist_tab = sd[j].hist_tab;
    if (jb.hist_tab) any_hist = true;
    jb.out_base = sd[j].out_base;
    jb.parts = (!jb.uncompressed && wants_parts(sd[j])) ? 1 : 0;
    // custom dictionary: its tail copies (kCDictMark records) beside the static words, whose
    // distances it shifts by its length (the decoder addresses it first, engine.ts:907-913);
    // a word's flagged distance must stay below 2^23, so words need a dictionary < 4 MiB
    if (!jb.uncompressed && sd[j].cdict) {
      jb.cdict = sd[j].cdict;
      jb.cdict_len = sd[j].cdict_len;
      jb.cdict_tail4 = sd[j].cdict_tail4;
      any_cdict = true;
    }
    jb.dict = (!jb.uncompressed && jb.cdict_len < (1u << 22) && !sd[j].streaming && !sd[j].hist_tab && prm.quality >= 10 && prm.lgwin <= 22 &&
               dict_enabled()) ? 1 : 0;
    jb.dict_span = dict_span();
    if (jb.dict) any_dict = true;
    if (jb.parts) any_parts = true;
    uint64_t idx_extra = 0;
    if (jb.parts) {
      jb.part_bits = part_bits();
      jb.part_lag = part_lag();
      const uint64_t nseg_j = (n + (1ull << jb.part_bits) - 1) >> jb.part_bits;
      jb.idx_payload = (uint32_t)(sizeof(PartHead) + nseg_j * sizeof(PartEntry));
      jb.idx_bits = part_index_bits(jb.hdr_lgwin ? window_bits_len((int)jb.hdr_lgwin) : 0, jb.idx_payload);
      idx_extra = jb.idx_payload + 16;
    }
    jb.pos_base = (uint32_t)pos_total;
    jb.seg_base = (uint32_t)segs.size();
    jb.mb_base = (uint32_t)mbs.size();
    if (!jb.uncompressed) {
      // metablock length: the reference's 16 MiB (MIB_MB_BITS: experiment knob, 2^18..2^24)
      static const uint64_t mb_max = 1ull << env_u32("MIB_MB_BITS", 24, kSegBits + 2, 24);
      for (uint64_t m0 = 0; m0 < n; m0 += mb_max) {
        Mb mb;
        memset(&mb, 0, sizeof(mb));
        mb.job = (uint32_t)j;
        mb.start = (uint32_t)m0;
        mb.end = (uint32_t)std::min<uint64_t>(n, m0 + mb_max);
        mb.first_seg = (uint32_t)segs.size();
        mb.is_last = (mb.end == n && jb.final_) ? 1 : 0;
        for (uint64_t s0 = m0; s0 < mb.end; s0 += kSeg) {
          Seg sg;
          memset(&sg, 0, sizeof(sg));
          sg.job = (uint32_t)j;
          sg.start = (uint32_t)s0;
          sg.end = (uint32_t)std::min<uint64_t>(mb.end, s0 + kSeg);
          sg.mb = (uint32_t)mbs.size();
          sg.cmd_off = (uint32_t)cmd_total;
          cmd_total += (sg.end - sg.start) / 2 + 4 + (2 << kMaxPieceShift);   // (room for the parse pieces' slices)
          // the segment's parse pieces: 2^shift of them from piece index npieces (Seg.pieces)
          const int pshift = dp_piece_shift(n, sd[j].streaming);
          sg.pieces = (uint32_t)(npieces << 3) | (uint32_t)pshift;
          npieces += 1ull << pshift;
          segs.push_back(sg);
        }
        mb.nseg = (uint32_t)segs.size() - mb.first_seg;
        mbs.push_back(mb);
      }
    }
    jb.nseg = (uint32_t)segs.size() - jb.seg_base;
    jb.nmb = (uint32_t)mbs.size() - jb.mb_base;
    const uint64_t span = ((n + kSeg - 1) / kSeg) * kSeg + kSeg;   // + a spare segment: end node, padding
    for (uint64_t q = 0; q < span / kSeg; q++) {
      seg_job.push_back((uint32_t)j);
      seg_ref.push_back(SegRef{jb.data - (uintptr_t)pos_total, (uint32_t)pos_total, (uint32_t)(pos_total + (jb.uncompressed ? 0 : n))});
    }
    pos_total += span;
    jb.out_off = out_scratch;
    jb.out_cap = n + n / 8 + 4096 + idx_extra;
    out_scratch += (jb.out_cap + 255) & ~255ull;
  }
  if (pos_total >= (1ull << 31)) return MIB_E_INVALID_ARG;
  const uint32_t total = (uint32_t)pos_total;
  const int nsegs = (int)segs.size(), nmbs = (int)mbs.size();
  int max_mb_units = 1, max_short_units = 1;   // (the split kernel's LDS: unit costs of the largest metablock)
  for (const Mb &mb : mbs) {
    const int nu = (int)mb.nseg * kSubPerSeg;
    max_mb_units = std::max(max_mb_units, nu);
    if (nu <= kSplitWideUnits) max_short_units = std::max(max_short_units, nu);
  }
  const size_t nm1 = std::max<size_t>(1, mbs.size()), ns1 = std::max<size_t>(1, segs.size());

  const size_t sort_tmp = sort_ws_bytes(total);
  size_t need = 64 * 256;
  need += 4 * (size_t)total * 4 + sort_tmp;
  need += (size_t)total * kMatchRec * 4;
  need += ((size_t)total + 1) * 8;
  need += cmd_total * (sizeof(RawCmd) + sizeof(Cmd) + 4);
  need += k * (sizeof(Job) + 1024 + 8) + ns1 * sizeof(Seg) + seg_job.size() * (4 + sizeof(SegRef)) + 256;
  need += nm1 * (sizeof(Mb) + sizeof(Codes) + kHdrBytes + kTreeSlots * kTreeBytes + 4 * (kLitSlots * 256 + kMaxBT * 704 + kMaxBT * kDistCtx * 128));
  need += ns1 * kSubPerSeg * (sizeof(Unit) + kSubHist * 4) + ns1 * kEmitTiles * 4;
  need += out_scratch + 64;
  need += ns1 * part_push_bytes();
  const bool two_pass = prm.quality >= 11 && zopfli_iterations() > 1;   // backward-references-hq.ts:562-605
  need += two_pass ? k * sizeof(CostModel) + cost_model_hist_bytes((int)k) : 0;
  need += std::max<uint64_t>(npieces, 1) * sizeof(Seg);   // parse pieces
  const bool cache = dp_cache(prm);
  need += cache ? dp_ring_hist_bytes((int)std::max<uint64_t>(npieces, (uint64_t)nsegs)) : 0;
  need += 41 * 256;   // alignment
  Workspace *ws = reinterpret_cast<Workspace *>(*ws_slot);
  if (!ws) {
    ws = new Workspace();
    *ws_slot = ws;
  }
  ws->need = std::max<uint64_t>(ws->need, need);
  if (ws->cap < need) {
    if (ws->buf) hipFree(ws->buf);
    ws->buf = nullptr;
    ws->cap = 0;
    const size_t c = need + need / 8;
    if (hipMalloc(&ws->buf, c) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    ws->cap = c;
  }
  Arena ar{ws->buf};
  uint32_t *keys = ar.take<uint32_t>(total), *vals = ar.take<uint32_t>(total);
  uint32_t *skeys = ar.take<uint32_t>(total), *svals = ar.take<uint32_t>(total);
  void *sort_ws = ar.take<uint8_t>(sort_tmp);
  uint32_t *matches = ar.take<uint32_t>((size_t)total * kMatchRec);
  uint64_t *choice = ar.take<uint64_t>((size_t)total + 1);
  RawCmd *raw = ar.take<RawCmd>(cmd_total);
  Cmd *cmds = ar.take<Cmd>(cmd_total);
  uint32_t *cmd_pos = ar.take<uint32_t>(cmd_total);
  Job *d_jobs = ar.take<Job>(k);
  Seg *d_segs = ar.take<Seg>(ns1);
  Mb *d_mbs = ar.take<Mb>(nm1);
  uint32_t *d_seg_job = ar.take<uint32_t>(seg_job.size());
  SegRef *d_seg_ref = ar.take<SegRef>(seg_ref.size());
  uint32_t *lit_h = ar.take<uint32_t>(k * 256);
  uint32_t *hl = ar.take<uint32_t>(nm1 * kLitSlots * 256);
  uint32_t *hc = ar.take<uint32_t>(nm1 * kMaxBT * 704);
  uint32_t *hd = ar.take<uint32_t>(nm1 * kMaxBT * kDistCtx * 128);
  Unit *units = ar.take<Unit>(ns1 * kSubPerSeg);
  uint32_t *tile_bits = ar.take<uint32_t>(ns1 * kEmitTiles);
  uint32_t *unit_h = ar.take<uint32_t>(ns1 * kSubPerSeg * kSubHist);
  Codes *codes = ar.take<Codes>(nm1);
  uint8_t *hdr = ar.take<uint8_t>(nm1 * kHdrBytes);
  uint8_t *trees = ar.take<uint8_t>(nm1 * kTreeSlots * kTreeBytes);
  uint64_t *d_dst_off = ar.take<uint64_t>(k + 2);   // (+ the pack's status)
  uint8_t *oscr = ar.take<uint8_t>(out_scratch + 64);
  PushSum *push = reinterpret_cast<PushSum *>(ar.take<uint8_t>(ns1 * part_push_bytes()));
  CostModel *model = two_pass ? ar.take<CostModel>(k) : nullptr;
  uint32_t *model_h = two_pass ? reinterpret_cast<uint32_t *>(ar.take<uint8_t>(cost_model_hist_bytes((int)k))) : nullptr;
  // iteration 1 of a two-pass parse only feeds the model: it parses the first
  // zopfli_sample() bytes of every segment (its own copy of the segment table)
  const bool sampled = two_pass && zopfli_sample() < kSeg;
  Seg *d_sample = sampled ? ar.take<Seg>(ns1) : nullptr;
  // the final parse on pieces of the segments (merge_pieces_kernel)
  const bool ps = npieces > (uint64_t)nsegs;
  Seg *d_pieces = ps ? ar.take<Seg>(std::max<uint64_t>(npieces, 1)) : nullptr;
  // the candidates' ring history (per DP lane group) and position words (in the sort's first
  // key buffer, free once the sort is done)
  uint32_t *ring_hist =
      cache ? reinterpret_cast<uint32_t *>(ar.take<uint8_t>(dp_ring_hist_bytes((int)std::max<uint64_t>(npieces, (uint64_t)nsegs)))) : nullptr;
  uint32_t *pos_words = cache ? keys : nullptr;
  uint32_t *d_any_binary = cache ? ar.take<uint32_t>(1) : nullptr;
  if (ar.off > ws->cap) return MIB_E_OUT_OF_MEMORY;

  Timer tm{ctx, st, mib_ctx_profiling(ctx) == 1, {}};   // (2: the decoder's kernels only)
  {   // the descriptors (jobs, segments, metablocks, position -> job / segment) lie back to back
      // in the arena (taken in that order): one upload of their image
    uint8_t *const d0 = reinterpret_cast<uint8_t *>(d_jobs);
    const size_t end = (size_t)(reinterpret_cast<uint8_t *>(d_seg_ref + seg_ref.size()) - d0);
    std::vector<uint8_t> img(end);
    auto put = [&](const void *dst, const void *src, size_t n) {
      if (n) memcpy(img.data() + (reinterpret_cast<const uint8_t *>(dst) - d0), src, n);
    };
    put(d_jobs, jobs.data(), sizeof(Job) * k);
    put(d_segs, segs.data(), sizeof(Seg) * nsegs);
    put(d_mbs, mbs.data(), sizeof(Mb) * nmbs);
    put(d_seg_job, seg_job.data(), seg_job.size() * 4);
    put(d_seg_ref, seg_ref.data(), seg_ref.size() * sizeof(SegRef));
    CK(hipMemcpyAsync(d0, img.data(), end, hipMemcpyHostToDevice, st));
  }
  // the sampled first iteration's and the parse pieces' segment tables, derived on the device
  // (the pieces' table of a C4 call is 12.6 MB: built on the host it was a host loop and a
  // pageable copy every call)
  if (nsegs) launch_derive_segs(st, d_segs, nsegs, sampled ? zopfli_sample() : 0u, d_sample, d_pieces);
  Seg *const d_fin = ps ? d_pieces : d_segs;   // the final parse's segment table
  const int nfin = ps ? (int)npieces : nsegs;
  CK(hipMemsetAsync(oscr, 0, out_scratch + 64, st));
  if (nsegs) {
    // lit_h, hl, hc, hd lie back to back in the arena (taken in that order): one memset
    CK(hipMemsetAsync(lit_h, 0, reinterpret_cast<uint8_t *>(hd + nm1 * kMaxBT * kDistCtx * 128) -
                                    reinterpret_cast<uint8_t *>(lit_h), st));
    CK(hipMemsetAsync(choice, 0, ((size_t)total + 1) * 8, st));
    const int depth = (int)env_u32("MIB_DEPTH", (uint32_t)depth_for_quality(prm.quality), 1, 64);   // override: experiments
    // (a batch of many metablocks fills the chip with each launch: there the independent
    // launches ran side by side were slower, C4 encode -1.8 %, r05ap)
    const DictDev *dd = any_dict ? dict_device(mib_ctx_device_of(ctx)) : nullptr;
    if (any_dict && !dd) return MIB_E_OUT_OF_MEMORY;   // (before the fork: nothing queued on the side stream yet)
    Fork fk = nmbs * 3 <= 256 ? fork_of(ws, st) : Fork{st, st, nullptr, nullptr};
    // every exit from here on (a failed launch check included) leaves st ordered after the side
    // stream's work, so the next call's memsets on st cannot overtake its kernels
    struct JoinAtExit {
      Fork &f;
      ~JoinAtExit() { f.join(); }
    } join_at_exit{fk};
    // the literal histogram and the context mode read only the input: beside the match search
    // (unforked, they keep their places after the match search: C4 encode -2 % with them first)
    const bool forked = fk.side != st;
    if (forked) {
      fk.fork();
      launch_lit_histo(fk.side, d_jobs, d_segs, nsegs, lit_h);
      launch_context_mode(fk.side, d_jobs, d_mbs, nmbs);
    }
    tm.start("bucket_sort");
    launch_sort(st, d_jobs, d_seg_job, (int)k, total, hash_bytes(prm), sort_ws, keys, vals, skeys, svals);
    tm.stop();
    tm.start("find_matches");
    launch_find_matches(st, d_jobs, d_seg_job, d_seg_ref, skeys, svals, total, depth, (1u << prm.lgwin) - 16, any_hist,
                        any_parts, matches);
    if (dd) launch_dict_matches(st, d_jobs, (int)k, dict_span(), dd->tab, dd->data, matches);
    if (any_cdict) launch_cdict_matches(st, d_jobs, d_seg_job, total, matches);
    if (near_scan(prm)) launch_near_matches(st, d_jobs, d_seg_job, d_seg_ref, total, (1u << prm.lgwin) - 16, any_hist, any_parts, matches);
    if (!forked) {
      if (any_hist) launch_hist_update(st, d_jobs, d_seg_job, skeys, svals, total);
      launch_lit_histo(st, d_jobs, d_segs, nsegs, lit_h);
    }
    // (the parse's candidates go by the metablocks' context modes)
    if (!forked) launch_context_mode(st, d_jobs, d_mbs, nmbs);
    tm.stop();
    fk.join();
    // (after the join: the words go by Job.binary, which the context modes set).  A call
    // whose metablocks are all UTF-8 text (C4, C2, C5) skips the candidates' inputs and build
    // altogether: its launch of that build would only wait for room on the chip beside the
    // other encode lane (an empty launch of the candidates' DP: +4.5 ms a C4 half batch, r06o)
    if (pos_words) {
      launch_any_binary(st, d_jobs, (int)k, d_any_binary);
      uint32_t any = 0;
      CK(hipMemcpyAsync(&any, d_any_binary, 4, hipMemcpyDeviceToHost, st));
      CK(hipStreamSynchronize(st));
      if (any) {
        launch_words(st, d_jobs, d_seg_job, d_seg_ref, total, pos_words);
      } else {
        pos_words = nullptr;
        ring_hist = nullptr;
      }
    }
    // the history table's update (read by the next call's match search): beside the parse
    fk.fork();
    if (forked && any_hist) launch_hist_update(fk.side, d_jobs, d_seg_job, skeys, svals, total);
    tm.start(two_pass ? "dp_sample" : "dp_parse");
    Seg *s1 = sampled ? d_sample : two_pass ? d_segs : d_fin;
    const int n1 = s1 == d_fin ? nfin : nsegs;
    launch_dp(st, d_jobs, s1, n1, lit_h, nullptr, matches, choice, any_cdict, prm.font, pos_words, ring_hist, d_mbs);
    tm.stop();
    tm.start("backtrack");
    launch_backtrack(st, d_jobs, s1, n1, choice, raw);
    tm.stop();
    if (two_pass) {   // iteration 2: prices from the first parse's commands
      tm.start("cost_model");
      launch_cost_model(st, d_jobs, (int)k, s1, nsegs, raw, model_h, model);
      tm.stop();
      tm.start("dp_parse");
      launch_dp(st, d_jobs, d_fin, nfin, lit_h, model, matches, choice, any_cdict, prm.font, pos_words, ring_hist, d_mbs);
      tm.stop();
      tm.start("backtrack");
      launch_backtrack(st, d_jobs, d_fin, nfin, choice, raw);
      tm.stop();
    }
    if (ps) launch_merge_pieces(st, d_jobs, d_segs, nsegs, d_pieces, raw);
    tm.start("codes");
    launch_carry(st, d_jobs, (int)k, d_segs, d_mbs);
    if (two_pass && rep_pass(prm)) launch_rep(st, d_jobs, d_segs, nsegs, model, raw, cmd_pos);   // (cmd_pos: scratch until codes)
    launch_ring_scan(st, d_jobs, (int)k, d_segs, nsegs, raw, push);
    launch_codes(st, d_jobs, d_segs, d_mbs, nsegs, raw, cmds, cmd_pos, units, unit_h);
    launch_dist_ring(st, d_jobs, (int)k, d_segs, cmds);
    tm.stop();
    tm.start("block_split");
    fk.fork();
    launch_split(st, fk.side, d_jobs, d_mbs, nmbs, units, unit_h, codes, max_mb_units, max_short_units);
    fk.join();
    tm.stop();
    tm.start("type_histo");
    launch_histo(st, d_jobs, d_segs, d_mbs, nsegs, cmds, cmd_pos, units, hl, hc, hd);
    tm.stop();
    tm.start("cluster");
    launch_cluster(st, d_jobs, d_mbs, nmbs, hl, hd);
    tm.stop();
    tm.start("huffman");
    fk.fork();
    launch_huffman(st, fk.side, d_jobs, d_mbs, nmbs, hl, hc, hd, codes, trees, hdr);
    fk.join();
    tm.stop();
    tm.start("sizes");
    launch_sizes(st, d_jobs, d_segs, d_mbs, nsegs, cmds, cmd_pos, codes, units, tile_bits);
    launch_offsets(st, d_jobs, (int)k, d_mbs, d_segs, oscr);
    tm.stop();
    tm.start("emit");
    launch_emit(st, d_jobs, d_mbs, nmbs, d_segs, nsegs, cmds, cmd_pos, codes, units, tile_bits, trees, hdr, oscr);
    tm.stop();
    tm.start("part_index");
    launch_part_index(st, d_jobs, (int)k, d_mbs, d_segs, nsegs, cmds, units, push, oscr);
    tm.stop();
  }
  tm.start("stored");
  launch_stored(st, d_jobs, (int)k, oscr);
  tm.stop();
  CK(hipGetLastError());
  // the streams' places in the packed output are summed on the device (dst_off_kernel), and
  // the jobs come back once, after the pack
  tm.start("pack");
  launch_pack(st, d_jobs, (int)k, out_pos, out_cap, d_dst_off, oscr, d_out);
  tm.stop();
  CK(hipGetLastError());
  uint64_t status = 0;
  CK(hipMemcpyAsync(jobs.data(), d_jobs, sizeof(Job) * k, hipMemcpyDeviceToHost, st));
  CK(hipMemcpyAsync(&status, d_dst_off + k + 1, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  CK(hipStreamSynchronize(st));
  if (status == 1) return MIB_E_NO_PROGRESS;   // cannot happen: offsets falls back first
  if (status) return MIB_E_NEED_SPACE;
  for (size_t j = 0; j < k; j++) {
    sizes[j] = (jobs[j].total_bits + 7) >> 3;
    if (dc_out)
      for (int q = 0; q < 4; q++) dc_out[j][q] = jobs[j].dc_out[q];
  }
  tm.collect();
  return 0;
}

// Workspace is ~72 bytes per position (keys 16, match records 32, choice 8, commands ~16).
// A call is split into as few groups as device memory allows -- one group when it fits, so
// no small tail group runs a whole parse at low occupancy -- below the 2^31 position limit
// of the 32-bit position indices.
constexpr uint64_t kWsBytesPerPosition = 80;
constexpr size_t kGroupStreams = 65536;   // bounds the per-call descriptor arrays

constexpr int kMaxLanes = 4;   // encode lanes at most (runtime.cpp kEncLanes; encode_streams)
uint64_t group_position_limit(mib_ctx *ctx) {
  size_t free_b = 0, total_b = 0;
  uint64_t lim = (1ull << 31) - 4 * (uint64_t)kSeg;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
    // (only the workspace a group grows is freed before it grows: the other lanes' stay held)
    const Workspace *ws = reinterpret_cast<const Workspace *>(*mib_ctx_enc_ws(ctx));
    const uint64_t held = ws ? ws->cap : 0;
    const uint64_t usable = ((uint64_t)free_b + held) / 10 * 8;   // leave 20% to the caller
    lim = std::min<uint64_t>(lim, std::max<uint64_t>(usable / kWsBytesPerPosition, 1ull << 24));
  }
  return lim;
}

// Encode lanes: a batch that fits one group runs as N parts (by positions) on N HIP streams at
// once, each with its own workspace, lanes 1.. driven from host threads of their own.  The
// parse and the match walk fill the chip on their own, but the ~20 small kernels after them
// (codes, split, clustering, Huffman, sizes, emit: ~50 ms of a C4 step) are latency-bound,
// block per segment or metablock: the other parts' kernels fill them.  Lanes 1.. pack their
// streams into staging buffers that are then copied behind lane 0's.  MIB_ENC_LANES (1-4).
uint64_t out_bound(uint64_t n);
constexpr uint64_t kLaneMinPositions = 32ull << 20;   // positions per lane at least
int enc_lanes() {
  static const int n = (int)env_u32("MIB_ENC_LANES", 2, 1, kMaxLanes);
  return n;
}
constexpr int kLaneStage = 4;   // mib_ctx_stage slots of lanes 1.. packed output: 4, 5, 6

// Split k streams into groups and encode them back to back into d_out.
int encode_streams(mib_ctx *ctx, const mib_enc_opts *o, const StreamDesc *sd, size_t k, uint8_t *d_out,
                   uint64_t out_cap, uint64_t *out_offsets, int32_t (*dc_out)[4], hipStream_t st) {
  const uint64_t kGroupPositions = group_position_limit(ctx);
  Params prm = make_params(o);
  out_offsets[0] = 0;
  // lanes when the whole call is one group
  uint64_t all = 0;
  for (size_t j = 0; j < k; j++) all += ((sd[j].n + kSeg - 1) / kSeg + 1) * kSeg;
  const int nl = (int)std::min<uint64_t>(std::min<uint64_t>((uint64_t)enc_lanes(), k), all / kLaneMinPositions);
  if (nl >= 2 && k <= kGroupStreams && all <= kGroupPositions) {
    // lane l takes streams [cut[l], cut[l + 1]): near equal positions
    std::vector<size_t> cut(nl + 1, k);
    cut[0] = 0;
    {
      uint64_t pos = 0;
      size_t j = 0;
      for (int l = 1; l < nl; l++) {   // (every lane gets a stream at least)
        while (j < k - (size_t)(nl - l) && (j <= cut[l - 1] || pos * nl < all * (uint64_t)l))
          pos += ((sd[j++].n + kSeg - 1) / kSeg + 1) * kSeg;
        cut[l] = j;
      }
    }
    std::vector<hipStream_t> lst(nl, st);
    std::vector<uint8_t *> lout(nl, d_out);
    std::vector<uint64_t> lcap(nl, out_cap);
    bool ok = true;
    for (int l = 1; l < nl && ok; l++) {
      uint64_t b = 64;
      for (size_t j = cut[l]; j < cut[l + 1]; j++) b += out_bound(sd[j].n);
      lst[l] = (hipStream_t)mib_ctx_lane_stream(ctx, l);
      lout[l] = mib_ctx_stage(ctx, kLaneStage + l - 1, b);
      lcap[l] = b;
      ok = lst[l] && lout[l];
    }
    if (ok) {
      // lanes 1.. start after everything already queued on st (inputs, the dictionary)
      hipEvent_t ev;
      CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      CK(hipEventRecord(ev, st));
      for (int l = 1; l < nl; l++) CK(hipStreamWaitEvent(lst[l], ev, 0));
      std::vector<uint64_t> sz(k, 0);
      std::vector<int> rc(nl, 0);
      const int dev = mib_ctx_device_of(ctx);
      auto run = [&](int l) {
        if (l && hipSetDevice(dev) != hipSuccess) {
          rc[l] = MIB_E_NO_DEVICE;
          return;
        }
        rc[l] = encode_group(ctx, prm, sd + cut[l], cut[l + 1] - cut[l], lout[l], lcap[l], 0, sz.data() + cut[l],
                             dc_out ? dc_out + cut[l] : nullptr, lst[l], l ? mib_ctx_lane_ws(ctx, l) : mib_ctx_enc_ws(ctx));
      };
      std::vector<std::thread> th;
      for (int l = 1; l < nl; l++) th.emplace_back(run, l);
      run(0);
      for (auto &t : th) t.join();
      hipEventDestroy(ev);
      for (int l = 0; l < nl; l++)
        if (rc[l]) return rc[l];
      for (size_t q = 0; q < k; q++) out_offsets[q + 1] = out_offsets[q] + sz[q];
      if (out_offsets[k] > out_cap) return MIB_E_NEED_SPACE;
      for (int l = 1; l < nl; l++) {
        const uint64_t n1 = out_offsets[cut[l + 1]] - out_offsets[cut[l]];
        if (n1) CK(hipMemcpyAsync(d_out + out_offsets[cut[l]], lout[l], n1, hipMemcpyDeviceToDevice, st));
      }
      CK(hipStreamSynchronize(st));
      return 0;
    }
  }
  size_t i = 0;
  std::vector<uint64_t> sizes;
  while (i < k) {
    size_t j = i;
    uint64_t pos = 0;
    while (j < k && j - i < kGroupStreams) {
      uint64_t span = ((sd[j].n + kSeg - 1) / kSeg + 1) * kSeg;
      if (j > i && pos + span > kGroupPositions) break;
      pos += span;
      j++;
    }
    sizes.assign(j - i, 0);
    int rc = encode_group(ctx, prm, sd + i, j - i, d_out, out_cap, out_offsets[i], sizes.data(), dc_out ? dc_out + i : nullptr,
                          st, mib_ctx_enc_ws(ctx));
    if (rc) return rc;
    for (size_t q = i; q < j; q++) out_offsets[q + 1] = out_offsets[q] + sizes[q - i];
    i = j;
  }
  return 0;
}

void fill_desc(StreamDesc &d, const uint8_t *p, uint64_t n, const Params &prm, bool one_shot) {
  d.d_data = p;
  d.n = n;
  d.final_ = 1;
  d.dc[0] = 4;
  d.dc[1] = 11;
  d.dc[2] = 15;
  d.dc[3] = 16;
  d.prev_bytes = 0;
  d.hist = 0;
  d.abs_base = 0;
  d.win_abs = 0;
  d.hist_tab = nullptr;
  d.out_base = 0;
  d.streaming = !one_shot;
  d.cdict = nullptr;
  d.cdict_len = 0;
  d.cdict_tail4 = 0;
  if (!one_shot) {
    d.hdr_lgwin = (uint32_t)prm.lgwin;
  } else if (n == 0) {
    d.hdr_lgwin = 10;   // encodeEmptyInput (encode.ts:92-103)
  } else if (prm.quality == 0 || n < 64) {   // encodeUncompressed (encode.ts:105-138)
    int lg = 10;
    if (n > 1) {
      int c = 0;
      while ((1ull << c) < n) c++;
      lg = std::max(10, std::min(24, c + 1));
    }
    d.hdr_lgwin = (uint32_t)lg;
  } else {
    d.hdr_lgwin = (uint32_t)prm.lgwin;
  }
}

// A custom dictionary (mib_enc_opts.dict) on the device.  Fewer than four bytes cannot hold
// a copy the encoder would emit (kCDictMark): no upload, no dictionary copies.
struct DevDict {
  uint8_t *d = nullptr;
  uint32_t n = 0, tail4 = 0;
  int upload(const uint8_t *h, uint64_t len, hipStream_t st) {
    if (!h || len < 4) return 0;
    if (len >= (1ull << 31)) return MIB_E_INVALID_ARG;
    if (hipMalloc(&d, len + 64) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    CK(hipMemcpyAsync(d, h, len, hipMemcpyHostToDevice, st));
    n = (uint32_t)len;
    tail4 = (uint32_t)h[len - 4] | ((uint32_t)h[len - 3] << 8) | ((uint32_t)h[len - 2] << 16) | ((uint32_t)h[len - 1] << 24);
    return 0;
  }
  void attach(StreamDesc &sd) const {
    sd.cdict = d;
    sd.cdict_len = n;
    sd.cdict_tail4 = tail4;
  }
  void release() {
    if (d) hipFree(d);
    d = nullptr;
    n = 0;
  }
};

constexpr uint64_t kMaxChunk = 256ull << 20;   // BrotliEncoder: the largest device encode it waits for
// BrotliEncoder: update() pieces up to half this size gather in a pinned host stage and reach
// the device one stage at a time (a copy call and its wait cost ~70 us: C5's 1 MiB pieces
// spent 80 ms of a 600 ms encode there); the stages of all encoders share a pinned budget
constexpr uint64_t kStage = 8ull << 20;
constexpr uint64_t kStageBudget = 256ull << 20;
std::atomic<uint64_t> g_stage_bytes{0};
std::atomic<int> g_live_encoders{0};   // BrotliEncoder objects alive (the default context keeps their workspace)
uint64_t out_bound(uint64_t n) { return n + n / 8 + 4096 + 16 + sizeof(PartHead) + ((n + kSeg - 1) / kSeg) * sizeof(PartEntry); }

}  // namespace

struct mib_encoder {
  mib_enc_opts opts;
  uint64_t pend = 0;              // input not yet encoded: on the device, at buf[cur] + hist
  bool started = false;
  bool finished = false;
  int32_t dc[4] = {4, 11, 15, 16};
  uint32_t prev_bytes = 0;        // the last two bytes handed to the engine (literal contexts)
  uint64_t window = 1 << 22;      // 2^lgwin: the history kept for the next chunk
  uint64_t block = 1 << 16;       // the reference's 2^lgblock (enc-constants.ts:129-147)
  uint64_t chunk = 0;             // input per device encode: whole blocks, at least this much --
                                  // 2^lgblock (the reference's cadence, encode.ts:366-374), or in
                                  // throughput mode (mib_enc_opts.stream_chunk) that many bytes,
                                  // growing with the stream (kMaxChunk)
  bool chunk_fixed = true;        // no growth (the reference's cadence; MIB_STREAM_CHUNK)
  // device state (the default context's device): the window of history, then the pending
  // input (update() copies each piece straight here), ping-ponged so the next chunk's history
  // is one device copy; the bucket table of earlier positions
  int device = -1;
  uint8_t *buf[2] = {nullptr, nullptr};
  uint64_t buf_cap = 0;
  int cur = 0;
  uint64_t hist = 0;              // history bytes at buf[cur][0, hist)
  uint64_t abs = 0;               // stream bytes encoded so far
  uint64_t obytes = 0;            // compressed bytes returned so far (part index offsets)
  uint32_t *tab = nullptr;
  std::vector<uint8_t> dict;      // customDictionary (the encoder's own copy) and its device copy
  DevDict ddict;
  uint8_t *stage = nullptr;       // small update() pieces gather here (pinned host memory) ...
  uint64_t staged = 0;            // ... these many bytes, still to go behind the pending input
};
extern "C" {

void mib_force_no_dp_cache(int off) { __atomic_store_n(&g_no_dp_cache, off ? 1 : 0, __ATOMIC_RELAXED); }

void mib_encode_ws_free(void *p) {
  Workspace *ws = reinterpret_cast<Workspace *>(p);
  if (!ws) return;
  if (ws->buf) hipFree(ws->buf);
  if (ws->side) hipStreamDestroy(ws->side);
  if (ws->fork_ev) hipEventDestroy(ws->fork_ev);
  if (ws->join_ev) hipEventDestroy(ws->join_ev);
  delete ws;
}
int mib_live_encoders(void) { return g_live_encoders.load(); }
// the default context after a host call: a workspace above `keep` bytes is released
void mib_encode_ws_trim(void **p, uint64_t keep) {   // (the hysteresis of runtime.cpp release_large)
  Workspace *ws = reinterpret_cast<Workspace *>(*p);
  if (!ws) return;
  ws->quiet = ws->need > keep ? 0 : ws->quiet + 1;
  ws->need = 0;
  if (ws->cap > keep && ws->quiet >= 4) {
    mib_encode_ws_free(ws);
    *p = nullptr;
  }
}

int mib_ctx_encode(mib_ctx *c, const mib_enc_opts *o, const uint8_t *d_in, const uint64_t *in_offsets, size_t k,
                   uint8_t *d_out, uint64_t out_cap, uint64_t *out_offsets, void *stream) {
  if (!c || !out_offsets || (k && (!d_in || !in_offsets || !d_out))) return MIB_E_INVALID_ARG;
  if (mib_ctx_ready(c) != 0) return MIB_E_NO_DEVICE;   // this context's device: gfx950 check, tables
  hipStream_t st = stream ? (hipStream_t)stream : (hipStream_t)mib_ctx_stream_of(c);
  mib_ctx_clear_times(c);
  Params prm = make_params(o);
  DevDict dd;
  int rc = o ? dd.upload(o->dict, o->dict_len, st) : 0;
  if (rc) return rc;
  std::vector<StreamDesc> sd(k);
  for (size_t i = 0; i < k; i++) {
    if (in_offsets[i + 1] < in_offsets[i] || in_offsets[i + 1] - in_offsets[i] >= (1ull << 31)) {
      dd.release();
      return MIB_E_INVALID_ARG;
    }
    fill_desc(sd[i], d_in + in_offsets[i], in_offsets[i + 1] - in_offsets[i], prm, true);
    dd.attach(sd[i]);
  }
  rc = encode_streams(c, o, sd.data(), k, d_out, out_cap, out_offsets, nullptr, st);
  hipStreamSynchronize(st);
  dd.release();
  return rc;
}

// host buffers -> device -> encode -> host
struct DefaultLock {   // the default context serves one host call at a time (runtime.cpp)
  DefaultLock() { mib_default_lock(1); }
  ~DefaultLock() { mib_default_lock(0); }
};

static int encode_host(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status) {
  DefaultLock use;
  mib_ctx *c = mib_default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  CK(hipSetDevice(mib_ctx_device_of(c)));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  Params prm = make_params(o);
  std::vector<uint64_t> ioff(k + 1, 0);
  uint64_t cap = 0;
  for (size_t i = 0; i < k; i++) {
    ioff[i + 1] = ioff[i] + ((in[i].size + 255) & ~(uint64_t)255);
    cap += out_bound(in[i].size);
  }
  // (the default context's staging buffers, kept across calls)
  uint8_t *d_in = mib_ctx_stage(c, 0, ioff[k] + 64), *d_out = mib_ctx_stage(c, 1, cap + 64);
  if (!d_in || !d_out) return MIB_E_OUT_OF_MEMORY;
  hipMemsetAsync(d_in, 0, ioff[k] + 64, st);
  std::vector<HostPiece> up;
  for (size_t i = 0; i < k; i++)
    if (in[i].size) up.push_back(HostPiece{d_in + ioff[i], in[i].data, in[i].size});
  int rc = ctx_upload(c, st, up.data(), up.size());   // (through the context's pinned ring)
  if (rc) return rc;
  DevDict dd;
  rc = o ? dd.upload(o->dict, o->dict_len, st) : 0;
  if (rc) return rc;
  std::vector<StreamDesc> sd(k);
  for (size_t i = 0; i < k; i++) {
    fill_desc(sd[i], d_in + ioff[i], in[i].size, prm, true);
    dd.attach(sd[i]);
  }
  std::vector<uint64_t> ooff(k + 1, 0);
  rc = encode_streams(c, o, sd.data(), k, d_out, cap, ooff.data(), nullptr, st);
  if (rc == 0) {
    std::vector<mib_buf *> outs(k);
    std::vector<const uint8_t *> src(k);
    std::vector<uint64_t> lens(k);
    for (size_t i = 0; i < k; i++) {
      outs[i] = &out[i];
      src[i] = d_out + ooff[i];
      lens[i] = ooff[i + 1] - ooff[i];
      if (status) status[i] = 0;
    }
    rc = mib_bufs_from_device(k, outs.data(), src.data(), lens.data());
  }
  hipStreamSynchronize(st);
  dd.release();
  return rc;
}

// The encoder's device buffers on the default context's device (dev), with room for
// `need` bytes of history + pending input (+ the zero tail the kernels read past a chunk).
static int encoder_room(mib_encoder *e, int dev, uint64_t need, hipStream_t st) {
  if (e->device >= 0 && e->device != dev) return MIB_E_INVALID_ARG;
  e->device = dev;
  need += 320;
  if (e->buf_cap < need) {   // first use, a grown chunk, or one large update()
    need = std::max(need, e->window + e->chunk + e->block + 320);
    uint8_t *nb[2] = {nullptr, nullptr};
    for (int b = 0; b < 2; b++)
      if (hipMalloc(&nb[b], need) != hipSuccess) {
        if (nb[0]) hipFree(nb[0]);
        return MIB_E_OUT_OF_MEMORY;
      }
    if (e->hist + e->pend) CK(hipMemcpyAsync(nb[0], e->buf[e->cur], e->hist + e->pend, hipMemcpyDeviceToDevice, st));
    CK(hipStreamSynchronize(st));
    for (int b = 0; b < 2; b++)
      if (e->buf[b]) hipFree(e->buf[b]);
    e->buf[0] = nb[0];
    e->buf[1] = nb[1];
    e->cur = 0;
    e->buf_cap = need;
  }
  if (!e->tab) {
    if (hipMalloc(&e->tab, sizeof(uint32_t) * kHistWays << kHashBits) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    CK(hipMemsetAsync(e->tab, 0xFF, sizeof(uint32_t) * kHistWays << kHashBits, st));
  }
  if (!e->ddict.d && e->dict.size() >= 4) {
    const int r = e->ddict.upload(e->dict.data(), e->dict.size(), st);
    if (r) return r;
  }
  return 0;
}

// The encoder's staged bytes -> its device buffer, behind the pending input.  The copy runs
// from pinned memory, asynchronously: the stage is reused only after the stream is synchronised.
static int flush_stage(mib_encoder *e, int dev, hipStream_t st) {
  if (!e->staged) return 0;
  const int rc = encoder_room(e, dev, e->hist + e->pend + e->staged, st);
  if (rc) return rc;
  CK(hipMemcpyAsync(e->buf[e->cur] + e->hist + e->pend, e->stage, e->staged, hipMemcpyHostToDevice, st));
  e->pend += e->staged;
  e->staged = 0;
  return 0;
}

// BrotliEncoder on the device: encoders es[0..k) (same options) each encode the first ns[i]
// bytes of their pending input in ONE launch sequence; outs[i] gets encoder i's bytes.  A
// chunk's matches reach the encoder's history (the last 2^lgwin bytes, kept in HBM) through
// the sorted chunk and the bucket table, so the stream is what a one-shot encode with the same
// window would produce, cut into chunks.  Caller: DefaultLock held, device current.
static int encoder_run(mib_ctx *c, mib_encoder *const *es, const uint64_t *ns, const bool *finals, size_t k,
                       mib_buf *const *outs) {
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  const Params prm = make_params(&es[0]->opts);
  uint64_t cap = 0;
  for (size_t i = 0; i < k; i++) cap += out_bound(ns[i]);
  uint8_t *d_out = mib_ctx_stage(c, 3, cap + 64);
  if (!d_out) return MIB_E_OUT_OF_MEMORY;
  std::vector<StreamDesc> sd(k);
  for (size_t i = 0; i < k; i++) {
    mib_encoder *e = es[i];
    uint8_t *base = e->buf[e->cur] + e->hist;
    // the input past this chunk moves to the other buffer (behind the history kept there),
    // and the chunk is followed by zeros, as a one-shot encode's input is
    const uint64_t keep = std::min<uint64_t>(e->window, e->hist + ns[i]);
    if (e->pend > ns[i])
      CK(hipMemcpyAsync(e->buf[e->cur ^ 1] + keep, base + ns[i], e->pend - ns[i], hipMemcpyDeviceToDevice, st));
    CK(hipMemsetAsync(base + ns[i], 0, 64, st));
    fill_desc(sd[i], base, ns[i], prm, false);
    sd[i].hdr_lgwin = e->started ? 0 : (uint32_t)prm.lgwin;
    sd[i].final_ = finals[i] ? 1 : 0;
    for (int q = 0; q < 4; q++) sd[i].dc[q] = e->dc[q];
    sd[i].prev_bytes = e->prev_bytes;
    sd[i].hist = (uint32_t)e->hist;
    sd[i].abs_base = (uint32_t)e->abs;
    sd[i].win_abs = (uint32_t)std::min<uint64_t>(e->abs, 1u << 24);
    sd[i].hist_tab = e->tab;
    sd[i].out_base = e->obytes;
    e->ddict.attach(sd[i]);
  }
  std::vector<uint64_t> ooff(k + 1, 0);
  std::vector<int32_t> dcs(4 * std::max<size_t>(k, 1));
  int rc = encode_streams(c, &es[0]->opts, sd.data(), k, d_out, cap, ooff.data(), (int32_t(*)[4])dcs.data(), st);
  if (rc) return rc;
  std::vector<const uint8_t *> src(k);
  std::vector<uint64_t> lens(k);
  std::vector<uint8_t> last(2 * k);   // each chunk's last two bytes (the next chunk's literal context)
  for (size_t i = 0; i < k; i++) {
    src[i] = d_out + ooff[i];
    lens[i] = ooff[i + 1] - ooff[i];
    const uint64_t m = std::min<uint64_t>(ns[i], 2);
    if (m) CK(hipMemcpyAsync(&last[2 * i + 2 - m], es[i]->buf[es[i]->cur] + es[i]->hist + ns[i] - m, m,
                             hipMemcpyDeviceToHost, st));
  }
  CK(hipStreamSynchronize(st));
  if ((rc = mib_bufs_from_device(k, outs, src.data(), lens.data()))) return rc;
  for (size_t i = 0; i < k; i++) {
    mib_encoder *e = es[i];
    const uint64_t n = ns[i];
    e->obytes += lens[i];
    for (int q = 0; q < 4; q++) e->dc[q] = dcs[4 * i + q];
    for (uint64_t q = 2 - std::min<uint64_t>(n, 2); q < 2; q++) e->prev_bytes = ((e->prev_bytes << 8) & 0xFF00) | last[2 * i + q];
    e->started = true;
    // the next chunk's history: the last 2^lgwin bytes, moved to the other buffer's front
    const uint64_t keep = std::min<uint64_t>(e->window, e->hist + n);
    if (keep)
      CK(hipMemcpyAsync(e->buf[e->cur ^ 1], e->buf[e->cur] + e->hist + n - keep, keep, hipMemcpyDeviceToDevice, st));
    e->cur ^= 1;
    e->hist = keep;
    e->abs += n;
    e->pend -= n;
    // a long stream gets longer device encodes: as much as it has already encoded, up to
    // kMaxChunk (a 32 MiB encode is 512 parse segments, a quarter of the DP's waves; C5's
    // 1 GiB stream takes 7 encodes instead of 32)
    if (!e->chunk_fixed) e->chunk = std::max(e->chunk, std::min<uint64_t>(kMaxChunk, e->abs / e->block * e->block));
  }
  // (no wait for the history moves: the next call's copies and launches are behind them on the
  // same stream, and a buffer is freed only by hipFree, which waits for the device)
  return 0;
}

int mib_encode(const uint8_t *in, size_t n, const mib_enc_opts *o, mib_buf *out) {
  if (!out || (!in && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  if (n >= (1ull << 31)) return MIB_E_INVALID_ARG;
  mib_span s{in, n};
  return encode_host(&s, 1, o, out, nullptr);
}

int mib_encode_batch(const mib_span *in, size_t k, const mib_enc_opts *o, mib_buf *out, int *status) {
  if (k && (!in || !out || !status)) return MIB_E_INVALID_ARG;
  for (size_t i = 0; i < k; i++) {
    out[i].data = nullptr;
    out[i].size = 0;
    status[i] = 0;
    if ((!in[i].data && in[i].size) || in[i].size >= (1ull << 31)) return MIB_E_INVALID_ARG;
  }
  if (!k) return 0;
  return encode_host(in, k, o, out, status);
}

// BrotliEncoder (encode.ts:290-409): input is taken in whole blocks of 2^lgblock
// (computeLgBlock, enc-constants.ts:129-147), at least `chunk` bytes per device encode; each
// encode ends in a byte-aligning empty metadata block so update() returns whole bytes.  The
// distance ring, the literal context and the 2^lgwin window of history carry over (the
// reference's ring, encode.ts:312-374, without Bug D's overwrite).
mib_encoder *mib_encoder_new(const mib_enc_opts *o) {
  if (o && o->dict && o->dict_len >= (1ull << 31)) return nullptr;
  mib_encoder *e = new mib_encoder();
  g_live_encoders++;
  if (o) e->opts = *o;
  else mib_enc_opts_default(&e->opts);
  if (o && o->dict && o->dict_len) e->dict.assign(o->dict, o->dict + o->dict_len);
  e->opts.dict = nullptr;   // (the caller's buffer is not kept)
  e->opts.dict_len = 0;
  Params prm = make_params(&e->opts);
  int lgblock;
  if (prm.quality == 0 || prm.quality == 1) lgblock = prm.lgwin;
  else if (prm.quality < 4) lgblock = 14;
  else {
    lgblock = 16;
    if (prm.quality >= 9 && prm.lgwin > lgblock) lgblock = std::min(18, prm.lgwin);
  }
  e->block = 1ull << lgblock;
  e->window = 1ull << prm.lgwin;
  // Output cadence.  Default: the reference's -- each update() encodes every complete block
  // it has, so a streaming caller gets bytes as soon as a block is complete.  stream_chunk:
  // throughput mode -- a device encode waits for that much input, and grows with what the
  // stream has already encoded (a 32 MiB encode is 512 parse segments, a quarter of the DP's
  // waves: small encodes leave the chip idle).  MIB_STREAM_CHUNK (MiB, tests and experiments):
  // a fixed size.
  if (knob("MIB_STREAM_CHUNK")) {
    e->chunk = (uint64_t)env_u32("MIB_STREAM_CHUNK", 32, 1, 4096) << 20;
    e->chunk_fixed = true;
  } else if (o && o->stream_chunk) {
    e->chunk = std::min<uint64_t>(o->stream_chunk, kMaxChunk);
    e->chunk_fixed = false;
  } else {
    e->chunk = e->block;
    e->chunk_fixed = true;
  }
  e->chunk = std::max<uint64_t>(e->block, e->chunk / e->block * e->block);
  return e;
}

static bool same_opts(const mib_enc_opts &a, const mib_enc_opts &b) {
  const Params x = make_params(&a), y = make_params(&b);
  return x.quality == y.quality && x.lgwin == y.lgwin && x.npostfix == y.npostfix && x.ndirect == y.ndirect;
}

int mib_encoder_update_batch(mib_encoder *const *es, const mib_span *in, size_t k, mib_buf *out) {
  if (k && (!es || !in || !out)) return MIB_E_INVALID_ARG;
  for (size_t i = 0; i < k; i++) {
    out[i].data = nullptr;
    out[i].size = 0;
    if (!es[i] || es[i]->finished || (!in[i].data && in[i].size)) return MIB_E_INVALID_ARG;
    for (size_t j = 0; j < i; j++)
      if (es[j] == es[i]) return MIB_E_INVALID_ARG;
  }
  DefaultLock use;
  mib_ctx *c = mib_default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  const int dev = mib_ctx_device_of(c);
  CK(hipSetDevice(dev));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  // a small piece that completes no chunk gathers in the encoder's stage; the others go
  // straight to its device buffer, behind the input already there
  bool copied = false;
  for (size_t i = 0; i < k; i++) {
    mib_encoder *e = es[i];
    const uint64_t n = in[i].size;
    int rc;
    if (n && n <= kStage / 2 && e->pend + e->staged + n < e->chunk) {
      if (!e->stage && g_stage_bytes.fetch_add(kStage) + kStage <= kStageBudget) {
        if (hipHostMalloc(&e->stage, kStage, hipHostMallocDefault) != hipSuccess) e->stage = nullptr;
      }
      if (!e->stage) g_stage_bytes.fetch_sub(kStage);   // (over budget / no pinned memory: no stage)
    }
    if (e->stage && n && n <= kStage / 2 && e->pend + e->staged + n < e->chunk) {
      if (e->staged + n > kStage) {   // a full stage goes to the device first
        if ((rc = flush_stage(e, dev, st))) return rc;
        CK(hipStreamSynchronize(st));
      }
      memcpy(e->stage + e->staged, in[i].data, n);
      e->staged += n;
      continue;
    }
    if ((rc = flush_stage(e, dev, st)) || (rc = encoder_room(e, dev, e->hist + e->pend + n, st))) return rc;
    if (n) CK(hipMemcpyAsync(e->buf[e->cur] + e->hist + e->pend, in[i].data, n, hipMemcpyHostToDevice, st));
    e->pend += n;
    copied = true;
  }
  if (copied) CK(hipStreamSynchronize(st));   // (the caller's buffers and the stages are free again)
  // encoders with a full chunk pending, grouped by options, one launch sequence per group
  std::vector<bool> done(k, false), ran(k, false);
  std::vector<mib_encoder *> run;
  std::vector<uint64_t> ns;
  std::vector<mib_buf *> outs;
  for (size_t i = 0; i < k; i++) {
    if (done[i]) continue;
    run.clear();
    ns.clear();
    outs.clear();
    for (size_t j = i; j < k; j++) {
      mib_encoder *e = es[j];
      if (done[j] || !same_opts(e->opts, es[i]->opts)) continue;
      done[j] = true;
      if (e->pend < e->chunk) continue;
      run.push_back(e);
      ns.push_back(e->pend / e->block * e->block);
      outs.push_back(&out[j]);
      ran[j] = true;
    }
    if (run.empty()) continue;
    std::unique_ptr<bool[]> fin(new bool[run.size()]());
    int rc = encoder_run(c, run.data(), ns.data(), fin.get(), run.size(), outs.data());
    if (rc) return rc;
  }
  for (size_t i = 0; i < k; i++) {   // the others: no bytes yet
    if (ran[i]) continue;
    int rc = mib_buf_from_device(&out[i], nullptr, 0);
    if (rc) return rc;
  }
  return 0;
}

int mib_encoder_update(mib_encoder *e, const uint8_t *in, size_t n, mib_buf *out) {
  if (!e || !out || (!in && n)) return MIB_E_INVALID_ARG;
  mib_span s{in, n};
  return mib_encoder_update_batch(&e, &s, 1, out);
}

int mib_encoder_finish(mib_encoder *e, mib_buf *out) {
  if (!e || !out) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  if (e->finished) return mib_buf_from_device(out, nullptr, 0);
  DefaultLock use;
  mib_ctx *c = mib_default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  const int dev = mib_ctx_device_of(c);
  CK(hipSetDevice(dev));
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(c);
  int rc;
  if ((rc = flush_stage(e, dev, st)) || (rc = encoder_room(e, dev, e->hist + e->pend, st))) return rc;
  const uint64_t n = e->pend;
  const bool fin = true;
  if ((rc = encoder_run(c, &e, &n, &fin, 1, &out))) return rc;
  e->finished = true;
  return 0;
}

void mib_encoder_free(mib_encoder *e) {
  if (!e) return;
  if (e->device >= 0) {
    hipSetDevice(e->device);
    for (int b = 0; b < 2; b++)
      if (e->buf[b]) hipFree(e->buf[b]);
    if (e->tab) hipFree(e->tab);
    e->ddict.release();
  }
  if (e->stage) {
    hipHostFree(e->stage);
    g_stage_bytes.fetch_sub(kStage);
  }
  delete e;
  g_live_encoders--;
}

}  // extern "C"
