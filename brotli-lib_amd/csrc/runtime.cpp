// brotli_amd host runtime: the C ABI of include/brotli_amd.h on top of the HIP kernels.
//
// Host work here is orchestration only -- argument handling mirroring decode.ts / encode.ts,
// header peeks, buffer sizing, H2D/D2H copies.  Every byte of encode/decode compute runs in
// the kernels (decode.hip, encode*.hip); with no gfx950 device the calls fail with
// MIB_E_NO_DEVICE rather than falling back to the CPU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "common.h"
#include "parts.h"

extern "C" hipError_t mib_decode_parts_launch(mib::DecJob *d_jobs, int njobs, uint8_t *d_scratch, uint64_t per_block,
                                              unsigned *d_ticket, int grid, int per_cu, hipStream_t stream);
extern "C" hipError_t mib_decode_launch(mib::DecJob *d_jobs, int njobs, uint8_t *d_scratch, uint64_t per_block,
                                        uint64_t ring_bytes, int grid, int per_cu, hipStream_t stream);
extern "C" hipError_t mib_decode_init_tables(const int16_t *host_lut);
extern "C" hipError_t mib_decode_peek_heads(const uint8_t *d_in, const uint64_t *d_offsets, int k, uint8_t *d_heads,
                                            hipStream_t stream);

const char *mib::knob(const char *name) {
#ifdef MIB_EXPERIMENTS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

namespace {
bool g_dev_unordered_any(int dev);
}
bool mib::lds_rank_ordered(int dev) { return !g_dev_unordered_any(dev); }

namespace {

#define HIP_OK(x)                               \
  do {                                          \
    hipError_t e_ = (x);                        \
    if (e_ != hipSuccess) return MIB_E_NO_DEVICE; \
  } while (0)

std::mutex g_mu;
int g_device = 0;                 // device of the default context (mib_init)
constexpr int kMaxDevices = 64;
bool g_dev_ready[kMaxDevices];    // per device: checked to be gfx950, command table uploaded
bool g_dev_unordered[kMaxDevices];  // per device: the LDS atomic order self-test failed
int g_dev_cus[kMaxDevices];       // per device: compute units

void build_cmd_lut(int16_t *lut) {   // engine.ts:65-90
  static const int ins_bits[24] = {0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 12, 14, 24};
  static const int copy_bits[24] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 7, 8, 9, 10, 24};
  int ins_off[24], copy_off[24];
  ins_off[0] = 0;
  copy_off[0] = 2;
  for (int i = 0; i < 23; i++) {
    ins_off[i + 1] = ins_off[i] + (1 << ins_bits[i]);
    copy_off[i + 1] = copy_off[i] + (1 << copy_bits[i]);
  }
  for (int c = 0; c < 704; c++) {
    int r = c >> 6, dco = -4;
    if (r >= 2) {
      r -= 2;
      dco = 0;
    }
    int ic = (((0x29850 >> (r * 2)) & 3) << 3) | ((c >> 3) & 7);
    int cc = (((0x26244 >> (r * 2)) & 3) << 3) | (c & 7);
    int co = copy_off[cc];
    lut[4 * c] = (int16_t)(ins_bits[ic] | (copy_bits[cc] << 8));
    lut[4 * c + 1] = (int16_t)ins_off[ic];
    lut[4 * c + 2] = (int16_t)co;
    lut[4 * c + 3] = (int16_t)(dco + std::min(co, 5) - 2);
  }
}

// Every device a context runs on is checked (gfx950) and gets its own copy of the decoder's
// __constant__ command table: module globals are per device.  Leaves `device` current.
int g_ndev = -1;   // visible devices, counted once (hipGetDeviceCount cost ~0.4 ms a call, r05m)
int ensure_device(int device) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_ndev <= 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return MIB_E_NO_DEVICE;
    g_ndev = n;
  }
  if (device < 0 || device >= g_ndev || device >= kMaxDevices) return MIB_E_NO_DEVICE;
  HIP_OK(hipSetDevice(device));
  if (g_dev_ready[device]) return 0;
  hipDeviceProp_t prop;
  HIP_OK(hipGetDeviceProperties(&prop, device));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fprintf(stderr, "brotli_amd: device %d is %s, this build targets gfx950\n", device, prop.gcnArchName);
    return MIB_E_NO_DEVICE;
  }
  g_dev_cus[device] = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  int16_t lut[704 * 4];
  build_cmd_lut(lut);
  HIP_OK(mib_decode_init_tables(lut));
  HIP_OK(hipDeviceSynchronize());
  const int64_t bad = mib_selftest_lds_atomic_order(4096);
  if (bad < 0) return MIB_E_NO_DEVICE;
  g_dev_unordered[device] = bad != 0;
  if (bad)
    fprintf(stderr, "brotli_amd: device %d serves returning LDS atomics out of lane order (%lld of 262144 lanes); "
                    "the bucket sort ranks by ballots\n", device, (long long)bad);
  g_dev_ready[device] = true;
  return 0;
}

int g_force_ballot = 0;
bool g_dev_unordered_any(int dev) {
  return __atomic_load_n(&g_force_ballot, __ATOMIC_RELAXED) || (dev >= 0 && dev < kMaxDevices && g_dev_unordered[dev]);
}

int ensure_init() {
  int dev;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    dev = g_device;
  }
  return ensure_device(dev);
}

// decodeWindowBits (engine.ts:91-124) on the first bits of a stream: sizes the ring scratch
int peek_window_bits(const uint8_t *b, size_t n) {
  uint32_t v = 0;
  for (size_t i = 0; i < 2 && i < n; i++) v |= (uint32_t)b[i] << (8 * i);
  if ((v & 1) == 0) return 16;
  int m = (v >> 1) & 7;
  if (m) return 17 + m;
  m = (v >> 4) & 7;
  if (m == 1) return 24;   // large window: rejected by the decoder, any ring size will do
  if (m) return 8 + m;
  return 17;
}

// ---------------------------------------------------------------- part index (parts.h)
// A stream's part plan: every valid entry of its index chain, in stream order.
struct PartPlan {
  std::vector<mib::PartEntry> ent;
  int64_t total = -1;
  int lgwin = 0;
};

// LSB-first bit reader over bytes fetched on demand (host memory or the device)
template <class Fetch>
struct HdrBits {
  Fetch &fetch;
  uint64_t bit;
  bool ok = true;
  uint32_t get(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++, bit++) {
      int byte = 0;
      if (!fetch(bit >> 3, 1, (uint8_t *)&byte)) {
        ok = false;
        return 0;
      }
      v |= (uint32_t)((byte >> (bit & 7)) & 1) << i;
    }
    return v;
  }
};

// The index block at byte `at` (with the stream's window bits first when at == 0).
// fetch(offset, length, dst) copies stream bytes; false past the end.
// *end: the byte after the block's payload (where the decoder reads the next header).
template <class Fetch>
bool read_part_index(Fetch &fetch, uint64_t at, PartPlan &plan, uint64_t *next, uint64_t *end) {
  HdrBits<Fetch> r{fetch, at * 8};
  if (at == 0) {   // decodeWindowBits (engine.ts:91-124)
    int lg;
    if (r.get(1) == 0) lg = 16;
    else {
      const int m = (int)r.get(3);
      if (m) lg = 17 + m;
      else {
        const int k = (int)r.get(3);
        if (k == 1) return false;
        lg = k ? 8 + k : 17;
      }
    }
    plan.lgwin = lg;
  }
  if (r.get(1) != 0 || r.get(2) != 3 || r.get(1) != 0) return false;   // ISLAST 0, metadata, reserved 0
  const int nb = (int)r.get(2);
  if (nb == 0) return false;
  const uint64_t len = (uint64_t)r.get(8 * nb) + 1;
  if (!r.ok || len < sizeof(mib::PartHead)) return false;
  const uint64_t pay = (r.bit + 7) >> 3;
  mib::PartHead h;
  if (!fetch(pay, sizeof(h), (uint8_t *)&h)) return false;
  if (h.magic != mib::kPartMagic || h.version != 1 || h.entry_bytes != sizeof(mib::PartEntry)) return false;
  if (sizeof(h) + (uint64_t)h.nentries * sizeof(mib::PartEntry) > len || h.nentries == 0 || h.nentries > (1u << 20)) return false;
  if (at == 0 && (int)h.lgwin != plan.lgwin) return false;
  std::vector<mib::PartEntry> e(h.nentries);
  if (!fetch(pay + sizeof(h), sizeof(mib::PartEntry) * e.size(), (uint8_t *)e.data())) return false;
  for (auto &x : e)
    if (x.flags & mib::kPartValid) plan.ent.push_back(x);
  plan.total = (int64_t)h.total;
  *next = h.next_byte;
  *end = pay + len;
  return true;
}

// The whole chain of a stream of n bytes; false if it has none or it does not hold together.
// Every part proves it ended exactly at the next entry's state, so the chain of parts is the
// serial decode once its FIRST entry is: that entry must be the metablock header the
// reference decoder reads right after skipping the first index block (its payload is opaque
// to every decoder, so an entry pointing into it -- or anywhere else -- is not trusted).
template <class Fetch>
bool plan_parts(Fetch &fetch, uint64_t n, PartPlan &plan) {
  uint64_t at = 0, next = 0, end = 0, first_end = 0;
  for (int guard = 0; guard < (1 << 16); guard++) {
    if (!read_part_index(fetch, at, plan, &next, &end)) {
      if (at == 0) return false;
      // BrotliEncoder.finish() with nothing pending adds only the final empty metablock
      // (ISLAST, ISLASTEMPTY: one byte 0x03): the chain is complete
      uint8_t b = 0;
      if (n - at == 1 && fetch(at, 1, &b) && b == 0x03) next = 0;
      break;
    }
    if (at == 0) first_end = end;
    if (next == 0) break;
    if (next <= at || next >= n) return false;
    at = next;
  }
  if (next != 0) return false;   // the stream's total is only known from the final chunk's head
  if (plan.ent.size() < 2 || plan.total <= 0 || plan.total > (1ll << 30)) return false;
  if (plan.ent[0].pos != 0 || !(plan.ent[0].flags & mib::kPartAtMb)) return false;
  if (plan.ent[0].bit != 8 * first_end || plan.ent[0].mb_bit != plan.ent[0].bit || plan.ent[0].mb_pos != 0) return false;
  for (size_t i = 0; i < plan.ent.size(); i++) {
    const mib::PartEntry &x = plan.ent[i];
    if (x.bit >= 8 * n || x.mb_bit > x.bit || x.mb_pos > x.pos || x.pos >= (uint64_t)plan.total) return false;
    if (i && (x.pos <= plan.ent[i - 1].pos || x.bit <= plan.ent[i - 1].bit)) return false;
  }
  return true;
}

struct HostFetch {   // stream bytes in host memory
  const uint8_t *b;
  uint64_t n;
  bool operator()(uint64_t off, uint64_t len, uint8_t *dst) const {
    if (off > n || len > n - off) return false;
    memcpy(dst, b + off, len);
    return true;
  }
};
// The first 16 bytes of a stream: window bits then an index block with our magic?
bool looks_indexed(const uint8_t *head, uint64_t n) {
  HostFetch f{head, std::min<uint64_t>(n, 16)};
  HdrBits<HostFetch> r{f, 0};
  if (r.get(1) != 0) {
    if (r.get(3) == 0 && r.get(3) == 1) return false;
  }
  if (r.get(1) != 0 || r.get(2) != 3 || r.get(1) != 0) return false;
  const int nb = (int)r.get(2);
  if (nb == 0) return false;
  r.get(8 * nb);
  const uint64_t pay = (r.bit + 7) >> 3;
  uint32_t magic = 0;
  return r.ok && f(pay, 4, (uint8_t *)&magic) && magic == mib::kPartMagic;
}

struct DeviceFetch {   // stream bytes on the device (small reads: index heads and entries)
  const uint8_t *d;
  uint64_t n;
  hipStream_t st;
  uint64_t cache_off = ~0ull;
  uint8_t cache[64] = {};
  bool operator()(uint64_t off, uint64_t len, uint8_t *dst) {
    if (off > n || len > n - off) return false;
    if (len == 1) {   // header bits: one cached 64-byte line at a time
      if (cache_off == ~0ull || off < cache_off || off >= cache_off + 64) {
        cache_off = off & ~63ull;
        const uint64_t m = std::min<uint64_t>(64, n - cache_off);
        if (hipMemcpyAsync(cache, d + cache_off, m, hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipStreamSynchronize(st) != hipSuccess)
          return false;
      }
      *dst = cache[off - cache_off];
      return true;
    }
    return hipMemcpyAsync(dst, d + off, len, hipMemcpyDeviceToHost, st) == hipSuccess && hipStreamSynchronize(st) == hipSuccess;
  }
};

// Waves a decode launch puts on each CU (1..4): a call with few streams gives each stream
// a whole CU's LDS (decode.hip decode_lds_plan)
int waves_per_cu(int device, size_t waves) {
  const size_t cus = (device >= 0 && device < kMaxDevices && g_dev_cus[device] > 0) ? (size_t)g_dev_cus[device] : 256;
  const size_t w = (waves + cus - 1) / cus;
  return (int)std::max<size_t>(1, std::min<size_t>(4, w));
}

}  // namespace

constexpr int kEncLanes = 4;                  // encode lanes at most (encode.hip)
constexpr int kStageSlots = 4 + kEncLanes - 1;   // + lanes 1.. packed output
struct mib_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  // decode scratch
  uint8_t *d_scratch = nullptr;
  uint64_t scratch_bytes = 0;
  mib::DecJob *d_jobs = nullptr;
  size_t jobs_cap = 0;
  uint8_t *d_aux = nullptr;   // small per-call staging (offsets, header peeks)
  uint64_t aux_bytes = 0;
  // part decoding: entries, positions, progress words, ticket (one allocation)
  uint8_t *d_parts = nullptr;
  uint64_t parts_bytes = 0;
  // encode workspaces (encode.hip): lane 0 on `stream`, lane l > 0 on lane_stream[l] (a batch
  // encode runs as concurrent parts, encode_streams)
  void *enc_ws = nullptr;
  void *lane_ws[kEncLanes] = {};
  hipStream_t lane_stream[kEncLanes] = {};
  // staging buffers of the host-memory entry points (input, output, dictionary, encoder
  // output) and lane 1's packed output, kept across calls so a small call does not pay
  // hipMalloc / hipFree
  uint8_t *stage[kStageSlots] = {};
  uint64_t stage_cap[kStageSlots] = {};
  // what the calls since the last trim needed of each buffer (trim's hysteresis, below)
  struct Trim {
    uint64_t need = 0;
    int quiet = 0;   // trims in a row whose calls needed no more than the keep size
  } stage_trim[kStageSlots], scratch_trim, parts_trim;
  // pinned host ring of the host <-> device transfers (host_io below): two halves, one filling
  // on the host while the other is in flight; allocated once, 2 x kRingHalf
  uint8_t *ring = nullptr;
  hipEvent_t ring_ev[2] = {nullptr, nullptr};
  bool ring_failed = false;
  // part decoding counters (streams decoded part-parallel / sent back to the serial decoder)
  uint64_t parts_used = 0, parts_fallback = 0;
  // profiling
  int profiling = 0;   // 0 off, 1 every kernel, 2 the decoder's only (mib_ctx_set_profiling)
  std::vector<mib_kernel_time> times;
  std::mutex times_mu;   // (two encode lanes collect at once)
  void add_time(const char *name, double ms) {
    std::lock_guard<std::mutex> lk(times_mu);
    for (auto &t : times)
      if (strncmp(t.name, name, sizeof(t.name)) == 0) {
        t.ms += ms;
        t.launches++;
        return;
      }
    mib_kernel_time t;
    memset(&t, 0, sizeof(t));
    strncpy(t.name, name, sizeof(t.name) - 1);
    t.ms = ms;
    t.launches = 1;
    times.push_back(t);
  }
};

extern "C" void mib_ctx_add_time(mib_ctx *c, const char *name, double ms) { c->add_time(name, ms); }
extern "C" int mib_ctx_profiling(mib_ctx *c) { return c->profiling; }
extern "C" void **mib_ctx_enc_ws(mib_ctx *c) { return &c->enc_ws; }
// encode lane l (1 .. kEncLanes - 1): its workspace slot, its stream (created on first use, on
// the context's device)
extern "C" void **mib_ctx_lane_ws(mib_ctx *c, int l) { return &c->lane_ws[l]; }
extern "C" void *mib_ctx_lane_stream(mib_ctx *c, int l) {
  if (!c->lane_stream[l]) {
    hipSetDevice(c->device);
    if (hipStreamCreateWithFlags(&c->lane_stream[l], hipStreamNonBlocking) != hipSuccess) c->lane_stream[l] = nullptr;
  }
  return (void *)c->lane_stream[l];
}
int grow(void **p, uint64_t *cap, uint64_t need);
// a staging buffer of at least `need` bytes (its content is not kept when it grows)
extern "C" uint8_t *mib_ctx_stage(mib_ctx *c, int slot, uint64_t need) {
  if (slot < 0 || slot >= kStageSlots) return nullptr;
  c->stage_trim[slot].need = std::max(c->stage_trim[slot].need, need);
  return grow((void **)&c->stage[slot], &c->stage_cap[slot], need) == 0 ? c->stage[slot] : nullptr;
}
extern "C" void mib_encode_ws_free(void *ws);

// ---------------------------------------------------------------- host <-> device transfers
// Host buffers cross PCIe through the context's pinned ring: the host copies a ring half while
// the other half is in flight, and host copies of more than a few MiB run on several threads.
// Pageable hipMemcpy of many 1 MiB results into fresh host memory ran at 0.5-2 GB/s and varied
// by 8x between runs; pinned halves move at PCIe speed, and the page faults
// of fresh result buffers are spread over the copy threads.
namespace {
constexpr uint64_t kRingHalf = 32ull << 20;
constexpr uint64_t kParCopyMin = 4ull << 20;   // below this, one thread copies
constexpr int kCopyThreads = 8;
using Piece = mib::HostPiece;
void par_copy(const std::vector<Piece> &ps) {
  uint64_t total = 0;
  for (const Piece &p : ps) total += p.n;
  const int nt = (int)std::min<uint64_t>(kCopyThreads, std::max<uint64_t>(1, total / kParCopyMin));
  auto run = [&](uint64_t lo, uint64_t hi) {   // bytes [lo, hi) of the concatenated pieces
    uint64_t at = 0;
    for (const Piece &p : ps) {
      const uint64_t a = std::max(lo, at), b = std::min(hi, at + p.n);
      if (a < b) memcpy(p.dst + (a - at), p.src + (a - at), b - a);
      at += p.n;
      if (at >= hi) break;
    }
  };
  if (nt <= 1) {
    run(0, total);
    return;
  }
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(run, total * t / nt, total * (t + 1) / nt);
  run(0, total / nt);
  for (auto &x : th) x.join();
}
bool ring_ready(mib_ctx *c) {
  if (c->ring) return true;
  if (c->ring_failed) return false;
  hipSetDevice(c->device);
  if (hipHostMalloc((void **)&c->ring, 2 * kRingHalf, hipHostMallocDefault) != hipSuccess) c->ring = nullptr;
  for (int h = 0; h < 2 && c->ring; h++)
    if (hipEventCreateWithFlags(&c->ring_ev[h], hipEventDisableTiming) != hipSuccess) {
      hipHostFree(c->ring);
      c->ring = nullptr;
    }
  if (!c->ring) c->ring_failed = true;
  return c->ring != nullptr;
}
// the pieces cut at ring-half boundaries: chunk j = the pieces' bytes [j H, (j + 1) H)
template <class F>
void for_chunks(const Piece *ps, size_t k, F fn) {
  std::vector<Piece> cur;
  uint64_t fill = 0;
  for (size_t i = 0; i < k; i++) {
    uint64_t off = 0;
    while (off < ps[i].n) {
      const uint64_t take = std::min(ps[i].n - off, kRingHalf - fill);
      cur.push_back(Piece{ps[i].dst + off, ps[i].src + off, take});
      off += take;
      fill += take;
      if (fill == kRingHalf) {
        fn(cur, fill);
        cur.clear();
        fill = 0;
      }
    }
  }
  if (fill) fn(cur, fill);
}
}  // namespace

// MIB_HOST_TIMING (experiment builds): each ring transfer's time waiting for the device and
// copying on the host, to stderr
namespace {
struct XferClock {
  const bool on = mib::knob("MIB_HOST_TIMING") != nullptr;
  const char *what;
  uint64_t bytes = 0;
  double wait_ms = 0, copy_ms = 0;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit XferClock(const char *w) : what(w) {}
  template <class F>
  void timed(double &acc, F fn) {
    if (!on) return fn();
    const auto a = std::chrono::steady_clock::now();
    fn();
    acc += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  }
  ~XferClock() {
    if (on)
      fprintf(stderr, "[mib] %s %.1f MiB: %.2f ms (device wait %.2f, host copy %.2f)\n", what, bytes / 1048576.0,
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(), wait_ms, copy_ms);
  }
};
}  // namespace
// host -> device: ps[i].src host, ps[i].dst device; asynchronous on st (returns once every
// source byte is in the ring: the caller may reuse its buffers)
int mib::ctx_upload(mib_ctx *c, void *stream, const HostPiece *ps, size_t k) {
  hipStream_t st = (hipStream_t)stream;
  uint64_t total = 0;
  for (size_t i = 0; i < k; i++) total += ps[i].n;
  if (total < kParCopyMin || !ring_ready(c)) {   // small: pageable copies
    for (size_t i = 0; i < k; i++)
      if (ps[i].n && hipMemcpyAsync(ps[i].dst, ps[i].src, ps[i].n, hipMemcpyHostToDevice, st) != hipSuccess) return MIB_E_NO_DEVICE;
    return 0;
  }
  int h = 0, rc = 0;
  XferClock clk("upload");
  clk.bytes = total;
  for_chunks(ps, k, [&](const std::vector<Piece> &ch, uint64_t) {
    if (rc) return;
    clk.timed(clk.wait_ms, [&] {   // the half's last copies are done
      if (hipEventSynchronize(c->ring_ev[h]) != hipSuccess) rc = MIB_E_NO_DEVICE;
    });
    if (rc) return;
    uint8_t *pin = c->ring + (uint64_t)h * kRingHalf;
    std::vector<Piece> hc;
    uint64_t po = 0;
    for (const Piece &p : ch) {
      hc.push_back(Piece{pin + po, p.src, p.n});
      po += p.n;
    }
    clk.timed(clk.copy_ms, [&] { par_copy(hc); });
    po = 0;
    for (const Piece &p : ch) {
      if (hipMemcpyAsync(p.dst, pin + po, p.n, hipMemcpyHostToDevice, st) != hipSuccess) { rc = MIB_E_NO_DEVICE; return; }
      po += p.n;
    }
    if (hipEventRecord(c->ring_ev[h], st) != hipSuccess) rc = MIB_E_NO_DEVICE;
    h ^= 1;
  });
  return rc;
}
// device -> host: ps[i].src device (written by work queued on st), ps[i].dst host; returns
// when every byte has arrived
int mib::ctx_download(mib_ctx *c, void *stream, const HostPiece *ps, size_t k) {
  hipStream_t st = (hipStream_t)stream;
  uint64_t total = 0;
  for (size_t i = 0; i < k; i++) total += ps[i].n;
  XferClock clk("download");
  clk.bytes = total;
  if (total < kParCopyMin || !ring_ready(c)) {
    for (size_t i = 0; i < k; i++)
      if (ps[i].n && hipMemcpyAsync(ps[i].dst, ps[i].src, ps[i].n, hipMemcpyDeviceToHost, st) != hipSuccess) return MIB_E_NO_DEVICE;
    return hipStreamSynchronize(st) == hipSuccess ? 0 : MIB_E_NO_DEVICE;
  }
  int h = 0, rc = 0;
  std::vector<Piece> pending;   // the previous chunk: ring -> host once its copies are done
  int ph = 0;
  auto drain = [&]() {
    if (pending.empty() || rc) return;
    clk.timed(clk.wait_ms, [&] {
      if (hipEventSynchronize(c->ring_ev[ph]) != hipSuccess) rc = MIB_E_NO_DEVICE;
    });
    if (rc) return;
    clk.timed(clk.copy_ms, [&] { par_copy(pending); });
    pending.clear();
  };
  for_chunks(ps, k, [&](const std::vector<Piece> &ch, uint64_t) {
    if (rc) return;
    uint8_t *pin = c->ring + (uint64_t)h * kRingHalf;
    std::vector<Piece> out;
    uint64_t po = 0;
    for (const Piece &p : ch) {
      if (hipMemcpyAsync(pin + po, p.src, p.n, hipMemcpyDeviceToHost, st) != hipSuccess) { rc = MIB_E_NO_DEVICE; return; }
      out.push_back(Piece{p.dst, pin + po, p.n});
      po += p.n;
    }
    if (hipEventRecord(c->ring_ev[h], st) != hipSuccess) { rc = MIB_E_NO_DEVICE; return; }
    drain();   // the other half, while this one is in flight
    pending = std::move(out);
    ph = h;
    h ^= 1;
  });
  drain();
  return rc;
}

namespace {

mib_ctx *g_default_ctx = nullptr;
// The host-buffer entry points (mib_encode / mib_decode / batches / BrotliEncoder) share the
// default context's stream and scratch: one call at a time (recursive: a batch decode retries
// a stream through mib_decode).
std::recursive_mutex g_default_mu;

mib_ctx *default_ctx() {
  if (ensure_init() != 0) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_default_ctx) {
    g_default_ctx = new mib_ctx();
    g_default_ctx->device = g_device;
    if (hipStreamCreateWithFlags(&g_default_ctx->stream, hipStreamNonBlocking) != hipSuccess) {
      delete g_default_ctx;
      g_default_ctx = nullptr;
    }
  }
  return g_default_ctx;
}

}  // namespace
int grow(void **p, uint64_t *cap, uint64_t need) {
  if (*cap >= need) return 0;
  if (*p) hipFree(*p);
  *p = nullptr;
  *cap = 0;
  uint64_t n = std::max<uint64_t>(need, 1 << 20);
  if (hipMalloc(p, n) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
  *cap = n;
  return 0;
}
namespace {
}  // namespace

extern "C" {

void mib_enc_opts_default(mib_enc_opts *o) {
  o->quality = 11;
  o->lgwin = 22;
  o->mode = MIB_MODE_GENERIC;
  o->size_hint = 0;
  o->dict = nullptr;
  o->dict_len = 0;
  o->stream_chunk = 0;
}

int mib_init(int device) {
  {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_default_ctx && device != g_device) return MIB_E_INVALID_ARG;   // the default context exists already
    g_device = device;
  }
  return ensure_init();
}

const char *mib_strerror(int code) {
  static thread_local char buf[96];
  if (code <= -1 && code >= -30) {
    snprintf(buf, sizeof(buf), "Brotli error code: %d", code);
    return buf;
  }
  switch (code) {
    case 0: return "ok";
    case MIB_E_NO_DEVICE: return "brotli_amd: no usable gfx950 (MI355X) device";
    case MIB_E_INVALID_ARG: return "brotli_amd: invalid argument";
    case MIB_E_OUT_OF_MEMORY: return "brotli_amd: out of device memory";
    case MIB_E_OUTPUT_LIMIT: return "Decompressed size exceeds limit";
    case MIB_E_NEED_SPACE: return "brotli_amd: output buffer too small";
    case MIB_E_JS_RANGE_ERROR: return "RangeError: offset is out of bounds";
    case MIB_E_JS_TYPE_ERROR: return "TypeError: Cannot read property 'subarray' of undefined";
    case MIB_E_NO_PROGRESS: return "brotli_amd: decoder made no progress";
  }
  snprintf(buf, sizeof(buf), "brotli_amd: error %d", code);
  return buf;
}

static mib_alloc_func g_alloc = nullptr;
static mib_free_func g_free = nullptr;
static void *g_opaque = nullptr;

void mib_set_allocator(mib_alloc_func alloc_func, mib_free_func free_func, void *opaque) {
  const bool both = alloc_func && free_func;
  g_alloc = both ? alloc_func : nullptr;
  g_free = both ? free_func : nullptr;
  g_opaque = both ? opaque : nullptr;
}

uint8_t *mib_buf_alloc(size_t n) {
  return (uint8_t *)(g_alloc ? g_alloc(g_opaque, n) : malloc(n ? n : 1));
}

int mib_buf_from_device(mib_buf *out, const void *d_src, uint64_t len) {
  out->data = mib_buf_alloc(len);
  out->size = 0;
  if (!out->data) return MIB_E_OUT_OF_MEMORY;
  out->size = len;
  // (called with the default context held: its stream produced d_src; large results go
  // through its pinned ring)
  mib_ctx *c = default_ctx();
  const mib::HostPiece p{out->data, (const uint8_t *)d_src, len};
  if (len && (!c || mib::ctx_download(c, c->stream, &p, 1) != 0)) {
    mib_buf_free(out);
    return MIB_E_NO_DEVICE;
  }
  return 0;
}

static int bufs_from_device(size_t k, mib_buf *const *outs, const uint8_t *const *d_src, const uint64_t *len);
// On failure no result stays allocated: a caller that reports the error keeps no buffer
// (the Python mirror's allocator would otherwise hold those bytes for the process' life)
int mib_bufs_from_device(size_t k, mib_buf *const *outs, const uint8_t *const *d_src, const uint64_t *len) {
  for (size_t i = 0; i < k; i++) outs[i]->data = nullptr, outs[i]->size = 0;
  const int rc = bufs_from_device(k, outs, d_src, len);
  if (rc)
    for (size_t i = 0; i < k; i++) mib_buf_free(outs[i]);
  return rc;
}
static int bufs_from_device(size_t k, mib_buf *const *outs, const uint8_t *const *d_src, const uint64_t *len) {
  if (!k) return 0;
  const uint8_t *lo = d_src[0], *hi = d_src[0];
  uint64_t sum = 0;
  for (size_t i = 0; i < k; i++) {
    lo = std::min(lo, d_src[i]);
    hi = std::max(hi, d_src[i] + len[i]);
    sum += len[i];
  }
  for (size_t i = 0; i < k; i++) {
    outs[i]->data = mib_buf_alloc(len[i]);
    outs[i]->size = 0;
    if (!outs[i]->data) return MIB_E_OUT_OF_MEMORY;
    outs[i]->size = len[i];
  }
  const uint64_t span = (uint64_t)(hi - lo);
  const bool sparse = span > 4 * sum + (1u << 20);
  // Large results on average (or scattered ones): through the default context's pinned ring,
  // straight into the result buffers, one device copy each.  Many small results in a dense
  // span: the span as ONE device copy (through the ring when large), then host copies out of
  // it -- a device copy call costs ~10 us, thousands of them would dominate.
  if (sparse || sum / k >= (256u << 10)) {
    mib_ctx *c = default_ctx();
    if (!c) return MIB_E_NO_DEVICE;
    std::vector<mib::HostPiece> ps;
    for (size_t i = 0; i < k; i++)
      if (len[i]) ps.push_back(mib::HostPiece{outs[i]->data, d_src[i], len[i]});
    return mib::ctx_download(c, c->stream, ps.data(), ps.size());
  }
  std::vector<uint8_t> host(span);
  if (span >= kParCopyMin) {
    mib_ctx *c = default_ctx();
    if (!c) return MIB_E_NO_DEVICE;
    const mib::HostPiece whole{host.data(), lo, span};
    if (mib::ctx_download(c, c->stream, &whole, 1) != 0) return MIB_E_NO_DEVICE;
  } else if (hipMemcpy(host.data(), lo, span, hipMemcpyDeviceToHost) != hipSuccess) {
    return MIB_E_NO_DEVICE;
  }
  std::vector<Piece> out;
  for (size_t i = 0; i < k; i++)
    if (len[i]) out.push_back(Piece{outs[i]->data, host.data() + (d_src[i] - lo), len[i]});
  par_copy(out);
  return 0;
}

void mib_buf_free(mib_buf *b) {
  if (b && b->data) {
    if (g_free) g_free(g_opaque, b->data);
    else free(b->data);
  }
  if (b) {
    b->data = nullptr;
    b->size = 0;
  }
}

int64_t mib_decoded_size(const uint8_t *b, size_t n) {   // engine.ts:2155-2192 (header parse only)
  size_t bp = 0;
  auto rb = [&](int k) {
    int v = 0;
    for (int i = 0; i < k; i++, bp++) {
      int byte = (bp >> 3) < n ? b[bp >> 3] : 0;
      v |= ((byte >> (bp & 7)) & 1) << i;
    }
    return v;
  };
  if (rb(1)) {
    int m = rb(3);
    if (m == 0) {
      int k = rb(3);
      if (k == 1) {
        if (rb(1)) return -1;
        rb(6);
      }
    }
  }
  int last = rb(1);
  if (last && rb(1)) return 0;
  int nib = rb(2) + 4;
  if (nib == 7) return -1;
  int64_t mlen = 0;
  for (int i = 0; i < nib; i++) mlen |= (int64_t)rb(4) << (i * 4);
  mlen++;
  return last ? mlen : -1;
}

mib_ctx *mib_ctx_new(int device) {
  if (ensure_device(device) != 0) return nullptr;
  mib_ctx *c = new mib_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  return c;
}

void mib_ctx_free(mib_ctx *c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->d_scratch) hipFree(c->d_scratch);
  if (c->d_jobs) hipFree(c->d_jobs);
  if (c->d_aux) hipFree(c->d_aux);
  if (c->d_parts) hipFree(c->d_parts);
  for (int i = 0; i < kStageSlots; i++)
    if (c->stage[i]) hipFree(c->stage[i]);
  if (c->enc_ws) mib_encode_ws_free(c->enc_ws);
  if (c->ring) hipHostFree(c->ring);
  for (int h = 0; h < 2; h++)
    if (c->ring_ev[h]) hipEventDestroy(c->ring_ev[h]);
  if (c->stream) hipStreamDestroy(c->stream);
  for (int l = 0; l < kEncLanes; l++) {
    if (c->lane_ws[l]) mib_encode_ws_free(c->lane_ws[l]);
    if (c->lane_stream[l]) hipStreamDestroy(c->lane_stream[l]);
  }
  delete c;
}

void mib_ctx_set_profiling(mib_ctx *c, int on) { c->profiling = on == 2 ? 2 : on != 0 ? 1 : 0; }

void mib_part_stats(mib_ctx *c, uint64_t *parallel, uint64_t *fallback) {
  if (!c) c = default_ctx();
  if (parallel) *parallel = c ? c->parts_used : 0;
  if (fallback) *fallback = c ? c->parts_fallback : 0;
}

// internal (encode.hip)
mib_ctx *mib_default_ctx(void) { return default_ctx(); }
// The host-memory entry points (here, encode.hip, woff2.hip) hold the default context for one
// call at a time; when the outermost of them returns, buffers a large call grew are released:
// a long-lived server keeps what its usual calls need (the latency path stays free of
// hipMalloc), not GiBs reserved since its largest call (a 1 GiB brotliDecode: a 1 GiB input
// stage and a 2 GiB output stage).
constexpr uint64_t kKeepStage = 64ull << 20;      // staging buffers (input, output, dictionary, encoder output)
constexpr uint64_t kKeepScratch = 1ull << 30;     // decoder scratch, part tables, encoder workspace
int g_default_depth = 0;                          // (guarded by g_default_mu)
extern "C" void mib_encode_ws_trim(void **ws, uint64_t keep);
extern "C" int mib_live_encoders(void);
// Hysteresis: a buffer above its keep size is released only once kQuietCalls trims in a row
// saw calls that needed no more than that -- a service whose every call is large keeps its
// buffers (a hipFree syncs the device and a fresh hipMalloc of GiBs costs more than the call:
// the r04 host-batch legs varied by 2 s from it), one large call among
// small ones gives its memory back a few calls later.
constexpr int kQuietCalls = 4;
static void release_large(uint8_t **p, uint64_t *cap, uint64_t keep, mib_ctx::Trim &tr) {
  tr.quiet = tr.need > keep ? 0 : tr.quiet + 1;
  tr.need = 0;
  if (*p && *cap > keep && tr.quiet >= kQuietCalls) {
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
  }
}
static void trim_default_ctx(mib_ctx *c) {
  hipSetDevice(c->device);
  // (while a BrotliEncoder lives, its chunk after chunk reuses the workspace and the encoder
  // output stage: kept)
  const bool streaming = mib_live_encoders() > 0;
  for (int i = 0; i < kStageSlots; i++)
    if (!(streaming && i == 3)) release_large(&c->stage[i], &c->stage_cap[i], kKeepStage, c->stage_trim[i]);
  release_large(&c->d_scratch, &c->scratch_bytes, kKeepScratch, c->scratch_trim);
  release_large(&c->d_parts, &c->parts_bytes, kKeepScratch, c->parts_trim);
  if (!streaming) {
    mib_encode_ws_trim(&c->enc_ws, kKeepScratch);
    for (int l = 0; l < kEncLanes; l++) mib_encode_ws_trim(&c->lane_ws[l], kKeepScratch);
  }
}
// a context's buffers above these sizes (staging slots; decoder scratch, part tables and
// encoder workspace), released (multi.cpp's shard contexts after each sharded call)
void mib_ctx_trim(mib_ctx *c, uint64_t keep_stage, uint64_t keep_scratch) {
  hipSetDevice(c->device);
  for (int i = 0; i < kStageSlots; i++) release_large(&c->stage[i], &c->stage_cap[i], keep_stage, c->stage_trim[i]);
  release_large(&c->d_scratch, &c->scratch_bytes, keep_scratch, c->scratch_trim);
  release_large(&c->d_parts, &c->parts_bytes, keep_scratch, c->parts_trim);
  mib_encode_ws_trim(&c->enc_ws, keep_scratch);
  for (int l = 0; l < kEncLanes; l++) mib_encode_ws_trim(&c->lane_ws[l], keep_scratch);
}
void mib_default_lock(int on) {
  if (on) {
    g_default_mu.lock();
    g_default_depth++;
  } else {
    if (--g_default_depth == 0 && g_default_ctx) trim_default_ctx(g_default_ctx);
    g_default_mu.unlock();
  }
}
namespace {
struct DefaultUse {   // mib_default_lock for this file's entry points
  DefaultUse() { mib_default_lock(1); }
  ~DefaultUse() { mib_default_lock(0); }
};
}  // namespace
int mib_ctx_ready(mib_ctx *c) { return c ? ensure_device(c->device) : MIB_E_INVALID_ARG; }
void *mib_ctx_stream_of(mib_ctx *c) { return (void *)c->stream; }
int mib_ctx_device_of(mib_ctx *c) { return c->device; }
void mib_ctx_clear_times(mib_ctx *c) { c->times.clear(); }

int mib_ctx_kernel_times(mib_ctx *c, mib_kernel_time *out, int max) {
  int n = std::min<int>(max, (int)c->times.size());
  for (int i = 0; i < n; i++) out[i] = c->times[i];
  return (int)c->times.size();
}

// decode k streams whose bytes are on the device; jobs[] describes them (host copy)
static int decode_jobs(mib_ctx *c, std::vector<mib::DecJob> &jobs, hipStream_t stream) {
  size_t k = jobs.size();
  if (k == 0) return 0;
  int max_log = 10;
  for (auto &j : jobs) max_log = std::max(max_log, j.max_ring_log);
  uint64_t ring_bytes = ((uint64_t)1 << max_log) + 37 + 256;
  ring_bytes = (ring_bytes + 255) & ~(uint64_t)255;
  uint64_t per_block = ring_bytes + mib::kDecodeTableInts * 4 + mib::kDecodeCtxBytes + 1152 + 1152 * 4 + 1100 * 4 + 3092 * 4;   // ... ctx-map table, block trees
  per_block = (per_block + 255) & ~(uint64_t)255;
  // (MIB_DEC_GRID: experiment knob, a smaller persistent grid -- fewer decoder waves per CU)
  static const size_t grid_cap = mib::knob("MIB_DEC_GRID") ? (size_t)std::max(1, atoi(mib::knob("MIB_DEC_GRID"))) : 2048;
  int grid = (int)std::min<size_t>(k, std::min<size_t>(grid_cap, 2048));
  int rc;
  c->scratch_trim.need = std::max(c->scratch_trim.need, per_block * (uint64_t)grid);
  if ((rc = grow((void **)&c->d_scratch, &c->scratch_bytes, per_block * (uint64_t)grid)) != 0) return rc;
  if (k > c->jobs_cap) {
    if (c->d_jobs) hipFree(c->d_jobs);
    c->d_jobs = nullptr;
    c->jobs_cap = 0;
    if (hipMalloc(&c->d_jobs, sizeof(mib::DecJob) * k) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    c->jobs_cap = k;
  }
  HIP_OK(hipMemcpyAsync(c->d_jobs, jobs.data(), sizeof(mib::DecJob) * k, hipMemcpyHostToDevice, stream));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->profiling) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, stream);
  }
  HIP_OK(mib_decode_launch(c->d_jobs, (int)k, c->d_scratch, per_block, ring_bytes, grid, waves_per_cu(c->device, (size_t)grid),
                           stream));
  if (c->profiling) hipEventRecord(e1, stream);
  HIP_OK(hipMemcpyAsync(jobs.data(), c->d_jobs, sizeof(mib::DecJob) * k, hipMemcpyDeviceToHost, stream));
  HIP_OK(hipStreamSynchronize(stream));
  if (c->profiling) {
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    c->add_time("decode_streams_kernel", ms);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  return 0;
}

// Decode indexed streams part-parallel.  streams[i] = (device input, length, device output,
// plan); ok[i] = 1 when every part of stream i checked out (its output is then complete:
// plan.total bytes), else the caller decodes it serially.
struct PartStream {
  const uint8_t *in;
  uint64_t in_len;
  uint8_t *out;
  const PartPlan *plan;
  const uint8_t *dict;   // customDictionary (device), or null
  uint64_t dict_len;
};
static int decode_parts(mib_ctx *c, const std::vector<PartStream> &ps, std::vector<int> &ok, hipStream_t stream) {
  size_t nj = 0, ne = 0;
  for (auto &p : ps) {
    nj += p.plan->ent.size();
    ne += p.plan->ent.size();
  }
  ok.assign(ps.size(), 0);
  if (nj == 0) return 0;
  // device layout: entries | positions (nparts + 1 per stream) | progress | ticket
  const uint64_t ent_b = ((ne * sizeof(mib::PartEntry)) + 255) & ~255ull;
  const uint64_t pos_b = (((ne + ps.size()) * 8) + 255) & ~255ull;
  const uint64_t prog_b = ((ne * 8) + 255) & ~255ull;
  int rc;
  c->parts_trim.need = std::max(c->parts_trim.need, ent_b + pos_b + prog_b + 256);
  if ((rc = grow((void **)&c->d_parts, &c->parts_bytes, ent_b + pos_b + prog_b + 256)) != 0) return rc;
  mib::PartEntry *d_ent = reinterpret_cast<mib::PartEntry *>(c->d_parts);
  int64_t *d_pos = reinterpret_cast<int64_t *>(c->d_parts + ent_b);
  uint64_t *d_prog = reinterpret_cast<uint64_t *>(c->d_parts + ent_b + pos_b);
  unsigned *d_ticket = reinterpret_cast<unsigned *>(c->d_parts + ent_b + pos_b + prog_b);
  std::vector<mib::PartEntry> ents;
  std::vector<int64_t> pos;
  std::vector<mib::DecJob> jobs;
  ents.reserve(ne);
  pos.reserve(ne + ps.size());
  jobs.reserve(nj);
  for (auto &p : ps) {
    const size_t e0 = ents.size(), p0 = pos.size();
    const size_t np = p.plan->ent.size();
    for (auto &x : p.plan->ent) {
      ents.push_back(x);
      pos.push_back((int64_t)x.pos);
    }
    pos.push_back(p.plan->total);
    for (size_t i = 0; i < np; i++) {
      mib::DecJob j;
      memset(&j, 0, sizeof(j));
      j.in = p.in;
      j.in_len = p.in_len;
      j.out = p.out;
      j.out_cap = (uint64_t)p.plan->total;
      j.out_size = p.plan->total;
      j.dict = p.dict;
      j.dict_len = p.dict_len;
      j.max_ring_log = p.plan->lgwin;
      j.part_entry = d_ent + e0 + i;
      j.next_entry = i + 1 < np ? d_ent + e0 + i + 1 : nullptr;
      j.ppos = d_pos + p0;
      j.prog = d_prog + e0;
      j.pidx = (int32_t)i;
      j.nparts = (int32_t)np;
      j.total = p.plan->total;
      jobs.push_back(j);
    }
  }
  uint64_t per_block = mib::kDecodeTableInts * 4 + mib::kDecodeCtxBytes + 1152 + 1152 * 4 + 1100 * 4 + 3092 * 4;
  per_block = (per_block + 255) & ~(uint64_t)255;
  static const size_t grid_cap = mib::knob("MIB_PART_GRID") ? (size_t)std::max(1, atoi(mib::knob("MIB_PART_GRID"))) : 2048;
  const int grid = (int)std::min<size_t>(nj, grid_cap);
  c->scratch_trim.need = std::max(c->scratch_trim.need, per_block * (uint64_t)grid);
  if ((rc = grow((void **)&c->d_scratch, &c->scratch_bytes, per_block * (uint64_t)grid)) != 0) return rc;
  if (nj > c->jobs_cap) {
    if (c->d_jobs) hipFree(c->d_jobs);
    c->d_jobs = nullptr;
    c->jobs_cap = 0;
    if (hipMalloc(&c->d_jobs, sizeof(mib::DecJob) * nj) != hipSuccess) return MIB_E_OUT_OF_MEMORY;
    c->jobs_cap = nj;
  }
  HIP_OK(hipMemcpyAsync(d_ent, ents.data(), sizeof(mib::PartEntry) * ne, hipMemcpyHostToDevice, stream));
  HIP_OK(hipMemcpyAsync(d_pos, pos.data(), 8 * pos.size(), hipMemcpyHostToDevice, stream));
  HIP_OK(hipMemsetAsync(d_prog, 0, prog_b + 256, stream));   // progress words and the ticket
  HIP_OK(hipMemcpyAsync(c->d_jobs, jobs.data(), sizeof(mib::DecJob) * nj, hipMemcpyHostToDevice, stream));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->profiling) {
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, stream);
  }
  HIP_OK(mib_decode_parts_launch(c->d_jobs, (int)nj, c->d_scratch, per_block, d_ticket, grid,
                                 waves_per_cu(c->device, (size_t)grid), stream));
  if (c->profiling) hipEventRecord(e1, stream);
  HIP_OK(hipMemcpyAsync(jobs.data(), c->d_jobs, sizeof(mib::DecJob) * nj, hipMemcpyDeviceToHost, stream));
  HIP_OK(hipStreamSynchronize(stream));
  if (c->profiling) {
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    c->add_time("decode_parts_kernel", ms);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
  }
  size_t q = 0;
  for (size_t i = 0; i < ps.size(); i++) {
    int good = 1;
    for (size_t k = 0; k < ps[i].plan->ent.size(); k++, q++)
      if (jobs[q].status != 0) good = 0;
    ok[i] = good;
  }
  c->parts_used += ps.size();
  for (int v : ok) c->parts_fallback += v ? 0 : 1;
  return 0;
}

int mib_ctx_decode(mib_ctx *c, const uint8_t *d_in, const uint64_t *in_offsets, size_t k, uint8_t *d_out,
                   const uint64_t *out_offsets, int64_t *out_sizes, int *status, void *stream) {
  if (!c || (k && (!d_in || !in_offsets || !d_out || !out_offsets))) return MIB_E_INVALID_ARG;
  if (ensure_device(c->device) != 0) return MIB_E_NO_DEVICE;
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  c->times.clear();
  std::vector<uint8_t> heads(16 * k + 16);
  std::vector<mib::DecJob> jobs(k);
  if (k) {   // window bits (and part index magic) of every stream, gathered in one launch
    int rc = grow((void **)&c->d_aux, &c->aux_bytes, (k + 1) * 8 + 16 * k + 256);
    if (rc) return rc;
    uint64_t *d_off = reinterpret_cast<uint64_t *>(c->d_aux);
    uint8_t *d_heads = c->d_aux + ((k + 1) * 8 + 255) / 256 * 256;
    HIP_OK(hipMemcpyAsync(d_off, in_offsets, (k + 1) * 8, hipMemcpyHostToDevice, st));
    HIP_OK(mib_decode_peek_heads(d_in, d_off, (int)k, d_heads, st));
    HIP_OK(hipMemcpyAsync(heads.data(), d_heads, 16 * k, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  }
  for (size_t i = 0; i < k; i++) {
    mib::DecJob &j = jobs[i];
    memset(&j, 0, sizeof(j));
    j.in = d_in + in_offsets[i];
    j.in_len = in_offsets[i + 1] - in_offsets[i];
    j.out = d_out + out_offsets[i];
    j.out_cap = out_offsets[i + 1] - out_offsets[i];
    j.out_size = -1;
    j.max_ring_log = peek_window_bits(&heads[16 * i], (size_t)std::min<uint64_t>(j.in_len, 2));
  }
  // streams with a part index decode part-parallel; the rest (and any part stream that does
  // not check out) one wave per stream
  std::vector<PartPlan> plans(k);
  std::vector<PartStream> ps;
  std::vector<size_t> ps_idx;
  std::vector<mib::DecJob> serial;
  std::vector<size_t> serial_idx;
  for (size_t i = 0; i < k; i++) {
    bool part = false;
    if (looks_indexed(&heads[16 * i], jobs[i].in_len)) {
      DeviceFetch f{jobs[i].in, jobs[i].in_len, st};
      part = plan_parts(f, jobs[i].in_len, plans[i]) && (uint64_t)plans[i].total + 64 <= jobs[i].out_cap;
    }
    if (part) {
      ps.push_back(PartStream{jobs[i].in, jobs[i].in_len, jobs[i].out, &plans[i], nullptr, 0});
      ps_idx.push_back(i);
    } else {
      serial.push_back(jobs[i]);
      serial_idx.push_back(i);
    }
  }
  std::vector<int> ok;
  int rc = decode_parts(c, ps, ok, st);
  if (rc) return rc;
  for (size_t q = 0; q < ps.size(); q++) {
    const size_t i = ps_idx[q];
    if (ok[q]) {
      jobs[i].status = 0;
      jobs[i].result_len = plans[i].total;
    } else {
      serial.push_back(jobs[i]);
      serial_idx.push_back(i);
    }
  }
  rc = decode_jobs(c, serial, st);
  if (rc) return rc;
  for (size_t q = 0; q < serial.size(); q++) jobs[serial_idx[q]] = serial[q];
  int worst = 0;
  for (size_t i = 0; i < k; i++) {
    out_sizes[i] = jobs[i].result_len;
    status[i] = jobs[i].status;
    if (jobs[i].status) worst = jobs[i].status;
  }
  return worst == MIB_E_NEED_SPACE ? MIB_E_NEED_SPACE : 0;
}

// one host stream through the device (brotliDecode semantics of decode.ts:18-65)
int mib_decode(const uint8_t *in, size_t n, const uint8_t *dict, size_t dict_n, int64_t max_out, int64_t exact_out,
               mib_buf *out) {
  if (!out || (!in && n)) return MIB_E_INVALID_ARG;
  out->data = nullptr;
  out->size = 0;
  DefaultUse use;
  mib_ctx *c = default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  hipSetDevice(c->device);
  int64_t out_size = -1;
  if (exact_out >= 0) {
    out_size = exact_out;   // legacy numeric signature: no peek (decode.ts:27-44)
  } else {
    int64_t est = mib_decoded_size(in, n);
    if (est > 0) out_size = est;
  }
  if (max_out >= 0 && out_size >= 0 && out_size > max_out) {
    out->size = (size_t)out_size;   // the size that exceeded the limit (decode.ts:46-50)
    return MIB_E_OUTPUT_LIMIT;
  }
  int known = out_size > 0;
  uint64_t cap = known ? (uint64_t)out_size : std::max<uint64_t>(1 << 20, 4 * (uint64_t)n + 4096);
  uint8_t *d_in = nullptr, *d_out = nullptr, *d_dict = nullptr;
  int rc = 0;
  if (!(d_in = mib_ctx_stage(c, 0, n + 16))) return MIB_E_OUT_OF_MEMORY;
  if (dict && !(d_dict = mib_ctx_stage(c, 2, dict_n + 16))) return MIB_E_OUT_OF_MEMORY;
  {
    const mib::HostPiece up[2] = {{d_in, in, n}, {d_dict, dict, dict ? dict_n : 0}};
    if ((rc = mib::ctx_upload(c, c->stream, up, dict ? 2 : 1))) return rc;
  }
  if (exact_out < 0) {   // a stream with a part index: part-parallel, checked
    PartPlan plan;
    HostFetch f{in, n};
    // (the index is untrusted: a total beyond maxOutputSize, or one the device cannot hold,
    // just leaves the stream to the serial decoder, which finds out what it really is)
    if (plan_parts(f, n, plan) && (max_out < 0 || plan.total <= max_out) &&
        (d_out = mib_ctx_stage(c, 1, (uint64_t)plan.total + 4096)) != nullptr) {
      std::vector<PartStream> ps(1);
      std::vector<int> ok;
      ps[0] = PartStream{d_in, n, d_out, &plan, d_dict, dict ? dict_n : 0};
      rc = decode_parts(c, ps, ok, c->stream);
      if (rc == 0 && ok[0]) {
        return mib_buf_from_device(out, d_out, (uint64_t)plan.total);
      }
      rc = 0;
    }
  }
  for (;;) {
    // room for the ring of a one-metablock stream (a power of two >= its size, + slack), so
    // the kernel can decode in place instead of through its scratch ring
    uint64_t alloc = 1;
    while (alloc < cap) alloc <<= 1;
    alloc += 4096;
    if (!(d_out = mib_ctx_stage(c, 1, alloc))) {
      rc = MIB_E_OUT_OF_MEMORY;
      break;
    }
    std::vector<mib::DecJob> jobs(1);
    mib::DecJob &j = jobs[0];
    memset(&j, 0, sizeof(j));
    j.in = d_in;
    j.in_len = n;
    j.out = d_out;
    j.out_cap = known ? alloc : cap;   // unknown size: cap is the growth step's limit
    j.out_size = known ? out_size : -1;
    j.dict = d_dict;
    j.dict_len = dict ? dict_n : 0;
    j.max_ring_log = peek_window_bits(in, n);
    rc = decode_jobs(c, jobs, c->stream);
    if (rc) break;
    rc = jobs[0].status;
    if (rc == MIB_E_NEED_SPACE && !known && cap < ((uint64_t)1 << 31)) {   // JS caps a Uint8Array near 2^31
      cap *= 4;
      continue;
    }
    if (rc == 0) {
      uint64_t len = (uint64_t)jobs[0].result_len;
      if (max_out >= 0 && (int64_t)len > max_out) {   // the header can lie about the size (decode.ts:57-62)
        out->size = len;
        rc = MIB_E_OUTPUT_LIMIT;
      } else {
        rc = mib_buf_from_device(out, d_out, len);
      }
    }
    break;
  }
  return rc;
}

int mib_decode_batch(const mib_span *in, size_t k, mib_buf *out, int *status) {
  static const bool timing = mib::knob("MIB_HOST_TIMING") != nullptr;
  const auto t_in = std::chrono::steady_clock::now();
  auto ms_since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_in).count(); };
  DefaultUse use;
  mib_ctx *c = default_ctx();
  if (!c) return MIB_E_NO_DEVICE;
  hipSetDevice(c->device);
  std::vector<uint64_t> ioff(k + 1, 0), ooff(k + 1, 0);
  for (size_t i = 0; i < k; i++) {
    ioff[i + 1] = ioff[i] + ((in[i].size + 255) & ~(size_t)255);
    int64_t est = mib_decoded_size(in[i].data, in[i].size);
    uint64_t cap = est > 0 ? (uint64_t)est : std::max<uint64_t>(1 << 16, 8 * (uint64_t)in[i].size);
    ooff[i + 1] = ooff[i] + ((cap + 64 + 255) & ~(uint64_t)255);
  }
  uint8_t *d_in = mib_ctx_stage(c, 0, ioff[k] + 16), *d_out = mib_ctx_stage(c, 1, ooff[k] + 64);
  if (!d_in || !d_out) return MIB_E_OUT_OF_MEMORY;
  int rc = 0;
  {
    std::vector<mib::HostPiece> up;
    for (size_t i = 0; i < k; i++)
      if (in[i].size) up.push_back(mib::HostPiece{d_in + ioff[i], in[i].data, in[i].size});
    if ((rc = mib::ctx_upload(c, c->stream, up.data(), up.size()))) return rc;
  }
  for (size_t i = 0; i < k; i++) out[i].data = nullptr, out[i].size = 0;
  // exact input lengths, padded slots
  std::vector<mib::DecJob> jobs(k);
  for (size_t i = 0; i < k; i++) {
    mib::DecJob &j = jobs[i];
    memset(&j, 0, sizeof(j));
    j.in = d_in + ioff[i];
    j.in_len = in[i].size;
    j.out = d_out + ooff[i];
    j.out_cap = ooff[i + 1] - ooff[i] - 64;
    int64_t est = mib_decoded_size(in[i].data, in[i].size);
    j.out_size = est > 0 ? est : -1;
    j.max_ring_log = peek_window_bits(in[i].data, in[i].size);
  }
  const double t_up = timing ? ms_since() : 0.0;
  rc = decode_jobs(c, jobs, c->stream);
  const double t_dec = timing ? ms_since() : 0.0;
  if (rc == 0) {
    std::vector<mib_buf *> outs;
    std::vector<const uint8_t *> src;
    std::vector<uint64_t> lens;
    for (size_t i = 0; i < k; i++) {
      status[i] = jobs[i].status;
      if (jobs[i].status == 0) {
        outs.push_back(&out[i]);
        src.push_back(d_out + ooff[i]);
        lens.push_back((uint64_t)jobs[i].result_len);
      }
    }
    if ((rc = mib_bufs_from_device(outs.size(), outs.data(), src.data(), lens.data()))) return rc;
    // then (the staging buffers are reused) the streams that outgrew their slots, alone
    // through the growing single-stream path
    for (size_t i = 0; i < k; i++)
      if (jobs[i].status == MIB_E_NEED_SPACE) status[i] = mib_decode(in[i].data, in[i].size, nullptr, 0, -1, -1, &out[i]);
  }
  if (timing)
    fprintf(stderr, "[mib] decode_batch %zu streams: upload done %.2f ms, decode done %.2f, results %.2f\n", k, t_up, t_dec,
            ms_since());
  return rc;
}

}  // extern "C"

extern "C" void mib_force_ballot_rank(int force) { __atomic_store_n(&g_force_ballot, force ? 1 : 0, __ATOMIC_RELAXED); }
// internal (multi.cpp): give back the context's pinned transfer ring (allocated again on the
// next large transfer)
extern "C" void mib_ctx_release_ring(mib_ctx *c) {
  if (!c || !c->ring) return;
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  hipHostFree(c->ring);
  c->ring = nullptr;
  for (int h = 0; h < 2; h++)
    if (c->ring_ev[h]) {
      hipEventDestroy(c->ring_ev[h]);
      c->ring_ev[h] = nullptr;
    }
}
