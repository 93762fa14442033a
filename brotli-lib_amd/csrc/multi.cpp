// brotli_amd: host batches sharded over several GPUs (SURVEY.md §8(b),(e): "batch calls are
// internally multi-GPU").  Independent buffers are assigned size-balanced to shards (the
// heaviest buffer to the least-loaded shard, like brotli_amd/shard.py), one host thread and
// one mib_ctx per shard; shard s runs on visible device s % device_count, so a one-GPU host
// can run two shards on one device (how the tests exercise the sharding).  Outputs come back
// in input order.  Nothing crosses between GPUs: the buffers are independent, so there is no
// collective; the results meet in host memory.
//
// A shard is a context plus its host-side staging, kept across calls in a pool (the same
// hygiene as the single-GPU host path, runtime.cpp): device input / output buffers are the
// context's staging slots (no hipMalloc / hipFree per call), the inputs are packed into a
// pinned host buffer and cross PCIe in ONE asynchronous copy per shard, and the results come
// back the same way (one copy per shard, then host copies into the result buffers) instead of
// one pageable hipMemcpy per buffer.  Concurrent sharded calls take different shards from the
// pool (created on demand), so they run side by side instead of queueing on one lock.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/brotli_amd.h"
#include "common.h"

// runtime.cpp: result buffers (mib_set_allocator's allocator), the context's stream and staging
extern "C" uint8_t *mib_buf_alloc(size_t n);
extern "C" void *mib_ctx_stream_of(mib_ctx *c);
extern "C" uint8_t *mib_ctx_stage(mib_ctx *c, int slot, uint64_t need);
extern "C" void mib_ctx_trim(mib_ctx *c, uint64_t keep_stage, uint64_t keep_scratch);
extern "C" void mib_ctx_release_ring(mib_ctx *c);

namespace {

constexpr int kMaxShards = 64;
// a shard's buffers above these sizes are released after the call (a batch of the usual size
// keeps its buffers; one huge batch does not pin GiBs of host and device memory forever)
constexpr uint64_t kKeepDevice = 4ull << 30;

int device_count() {   // (a hipGetDeviceCount costs ~0.4 ms: a positive count is kept, a failure is retried)
  static std::atomic<int> known{0};
  int n = known.load(std::memory_order_relaxed);
  if (n > 0) return n;
  int c = 0;
  n = hipGetDeviceCount(&c) == hipSuccess ? c : 0;
  if (n > 0) known.store(n, std::memory_order_relaxed);
  return n;
}

// A shard: its own context (stream, device buffers, pinned transfer ring: runtime.cpp)
struct Shard {
  int device = -1;
  mib_ctx *ctx = nullptr;
  void trim() { mib_ctx_trim(ctx, kKeepDevice, kKeepDevice); }
};

std::mutex g_pool_mu;                        // guards the free lists only
std::vector<Shard *> g_pool[kMaxShards];     // idle shards for shard index s (device s % n)

Shard *acquire(int s, int dev) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (!g_pool[s].empty()) {
      Shard *sh = g_pool[s].back();
      g_pool[s].pop_back();
      return sh;
    }
  }
  mib_ctx *c = mib_ctx_new(dev);
  if (!c) return nullptr;
  Shard *sh = new Shard();
  sh->device = dev;
  sh->ctx = c;
  return sh;
}
// At most kKeepIdle idle shards per index stay pooled (each holds a context with up to
// kKeepDevice per buffer and its 64 MiB pinned transfer ring); a burst of concurrent sharded
// calls destroys its extra shards as they finish instead of keeping them for the process's
// life.  Only the first shard of each device keeps its ring while pooled: shard indices past
// the device count (several shards on one device) give it back, so the pool pins at most one
// ring per device however many shards a call asked for.
constexpr size_t kKeepIdle = 1;
void release(int s, Shard *sh) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (g_pool[s].size() < kKeepIdle) {
      sh->trim();
      if (s >= device_count()) mib_ctx_release_ring(sh->ctx);
      g_pool[s].push_back(sh);
      return;
    }
  }
  mib_ctx_free(sh->ctx);
  delete sh;
}

// size-balanced assignment: buffers by size, largest first, each to the least-loaded shard
std::vector<std::vector<size_t>> assign(const mib_span *in, size_t k, int shards) {
  std::vector<size_t> order(k);
  for (size_t i = 0; i < k; i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return in[a].size > in[b].size; });
  std::vector<std::vector<size_t>> out(shards);
  std::vector<uint64_t> load(shards, 0);
  for (size_t i : order) {
    const int s = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    out[s].push_back(i);
    load[s] += in[i].size + 64;
  }
  for (auto &v : out) std::sort(v.begin(), v.end());   // each shard keeps input order
  return out;
}

uint64_t align256(uint64_t n) { return (n + 255) & ~255ull; }

// The shard's inputs packed back to back (the device-resident ABI reads stream i from
// [in_offsets[i], in_offsets[i + 1])) into device staging slot 0 through the shard context's
// pinned ring, 64 zero bytes after the last.
int upload(Shard &sh, const mib_span *in, const std::vector<size_t> &idx, std::vector<uint64_t> &ioff, uint8_t **d_in,
           hipStream_t st) {
  const size_t k = idx.size();
  ioff.assign(k + 1, 0);
  for (size_t q = 0; q < k; q++) ioff[q + 1] = ioff[q] + in[idx[q]].size;
  *d_in = mib_ctx_stage(sh.ctx, 0, ioff[k] + 64);
  if (!*d_in) return MIB_E_OUT_OF_MEMORY;
  std::vector<mib::HostPiece> ps;
  for (size_t q = 0; q < k; q++)
    if (in[idx[q]].size) ps.push_back(mib::HostPiece{*d_in + ioff[q], in[idx[q]].data, in[idx[q]].size});
  if (hipMemsetAsync(*d_in + ioff[k], 0, 64, st) != hipSuccess) return MIB_E_NO_DEVICE;
  return mib::ctx_upload(sh.ctx, st, ps.data(), ps.size());
}

// Results [d_src[q], + len[q]) on the device -> out[idx[q]]: allocated, then copied through
// the shard context's pinned ring.
int download(Shard &sh, const std::vector<size_t> &idx, const std::vector<const uint8_t *> &d_src,
             const std::vector<uint64_t> &len, const std::vector<bool> &want, mib_buf *out, hipStream_t st) {
  const size_t k = idx.size();
  std::vector<mib::HostPiece> ps;
  for (size_t q = 0; q < k; q++) {
    if (!want[q]) continue;
    mib_buf &o = out[idx[q]];
    o.data = mib_buf_alloc(len[q]);
    o.size = 0;
    if (!o.data) return MIB_E_OUT_OF_MEMORY;
    o.size = len[q];
    if (len[q]) ps.push_back(mib::HostPiece{o.data, d_src[q], len[q]});
  }
  return mib::ctx_download(sh.ctx, st, ps.data(), ps.size());
}

int encode_shard(Shard &sh, const mib_span *in, const std::vector<size_t> &idx, const mib_enc_opts *o, mib_buf *out,
                 int *status) {
  const size_t k = idx.size();
  if (!k) return 0;
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(sh.ctx);
  std::vector<uint64_t> ioff, ooff(k + 1, 0);
  uint8_t *d_in = nullptr;
  int rc;
  if ((rc = upload(sh, in, idx, ioff, &d_in, st))) return rc;
  uint64_t cap = 0;
  for (size_t q = 0; q < k; q++) {
    const uint64_t n = in[idx[q]].size;
    cap += n + n / 8 + 8192 + ((n >> 16) + 1) * 72;   // (the encoder's bound: stored blocks + a part index)
  }
  uint8_t *d_out = mib_ctx_stage(sh.ctx, 1, cap + 64);
  if (!d_out) return MIB_E_OUT_OF_MEMORY;
  if ((rc = mib_ctx_encode(sh.ctx, o, d_in, ioff.data(), k, d_out, cap, ooff.data(), st))) return rc;
  std::vector<const uint8_t *> src(k);
  std::vector<uint64_t> lens(k);
  std::vector<bool> want(k, true);
  for (size_t q = 0; q < k; q++) {
    src[q] = d_out + ooff[q];
    lens[q] = ooff[q + 1] - ooff[q];
    status[idx[q]] = 0;
  }
  return download(sh, idx, src, lens, want, out, st);
}

int decode_shard(Shard &sh, const mib_span *in, const std::vector<size_t> &idx, mib_buf *out, int *status) {
  const size_t k = idx.size();
  if (!k) return 0;
  hipStream_t st = (hipStream_t)mib_ctx_stream_of(sh.ctx);
  std::vector<uint64_t> ioff, ooff(k + 1, 0);
  for (size_t q = 0; q < k; q++) {
    const mib_span &s = in[idx[q]];
    const int64_t est = mib_decoded_size(s.data, s.size);
    // a header size, else room for a part-indexed stream's total (known only from its index),
    // else 8x the input; a stream that outgrows it is decoded again alone
    const uint64_t capq = est > 0 ? (uint64_t)est : std::max<uint64_t>(1 << 16, 8 * (uint64_t)s.size);
    ooff[q + 1] = ooff[q] + align256(capq + 4096);
  }
  uint8_t *d_in = nullptr;
  int rc;
  static const bool timing = mib::knob("MIB_HOST_TIMING") != nullptr;
  const auto t_in = std::chrono::steady_clock::now();
  auto ms_since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_in).count(); };
  if ((rc = upload(sh, in, idx, ioff, &d_in, st))) return rc;
  uint8_t *d_out = mib_ctx_stage(sh.ctx, 1, ooff[k] + 64);
  if (!d_out) return MIB_E_OUT_OF_MEMORY;
  std::vector<int64_t> sizes(k);
  std::vector<int> stv(k);
  const double t_up = timing ? ms_since() : 0.0;
  rc = mib_ctx_decode(sh.ctx, d_in, ioff.data(), k, d_out, ooff.data(), sizes.data(), stv.data(), st);
  if (timing) fprintf(stderr, "[mib] shard %d: %zu streams, upload done %.2f ms, decode done %.2f\n", sh.device, k, t_up, ms_since());
  if (rc && rc != MIB_E_NEED_SPACE) return rc;
  std::vector<const uint8_t *> src(k);
  std::vector<uint64_t> lens(k);
  std::vector<bool> want(k);
  for (size_t q = 0; q < k; q++) {
    status[idx[q]] = stv[q];
    want[q] = stv[q] == 0;
    src[q] = d_out + ooff[q];
    lens[q] = want[q] ? (uint64_t)sizes[q] : 0;
  }
  if ((rc = download(sh, idx, src, lens, want, out, st))) return rc;
  for (size_t q = 0; q < k; q++)
    if (stv[q] == MIB_E_NEED_SPACE)   // the growing single-stream path
      status[idx[q]] = mib_decode(in[idx[q]].data, in[idx[q]].size, nullptr, 0, -1, -1, &out[idx[q]]);
  return 0;
}

// mib_force_shards (tests): the shard path even on one device, so a one-GPU box exercises it
int g_force_shards = 0;
bool force_shards() { return __atomic_load_n(&g_force_shards, __ATOMIC_RELAXED) != 0; }

// run fn(shard, indices) on `shards` host threads; the first error wins.  per_device: at most
// one shard per device, a device's streams in one call (the decoder: four 256-stream shards on
// one GPU left one shard's kernel queued behind the others' on a shared hardware queue, 298 vs
// 159 ms, r05u -- the call ~25 % slower than one launch of all 1,024)
template <class F>
int run_shards(const mib_span *in, size_t k, int n_gpus, F fn, bool per_device = false) {
  const int ndev = device_count();
  if (ndev <= 0) return MIB_E_NO_DEVICE;
  int shards = n_gpus <= 0 ? ndev : n_gpus;
  if (per_device) shards = std::min(shards, ndev);
  shards = std::max(1, std::min<int>({shards, kMaxShards, (int)std::max<size_t>(k, 1)}));
  std::vector<Shard *> sh(shards, nullptr);
  int rc = 0;
  for (int s = 0; s < shards && !rc; s++)
    if (!(sh[s] = acquire(s, s % ndev))) rc = MIB_E_NO_DEVICE;
  if (!rc) {
    const std::vector<std::vector<size_t>> parts = assign(in, k, shards);
    std::vector<int> rcs(shards, 0);
    std::vector<std::thread> th;
    for (int s = 0; s < shards; s++)
      th.emplace_back([&, s] {
        hipSetDevice(sh[s]->device);
        rcs[s] = fn(*sh[s], parts[s]);
      });
    for (auto &t : th) t.join();
    for (int r : rcs)
      if (r && !rc) rc = r;
  }
  for (int s = 0; s < shards; s++)
    if (sh[s]) release(s, sh[s]);
  return rc;
}

}  // namespace

extern "C" {

int mib_encode_batch_n(const mib_span *in, size_t k, const mib_enc_opts *o, int n_gpus, mib_buf *out, int *status) {
  if (k && (!in || !out || !status)) return MIB_E_INVALID_ARG;
  for (size_t i = 0; i < k; i++) {
    out[i].data = nullptr;
    out[i].size = 0;
    status[i] = 0;
    if ((!in[i].data && in[i].size) || in[i].size >= (1ull << 31)) return MIB_E_INVALID_ARG;
  }
  if (!k) return 0;
  // one device (or one shard asked for): the one-context call -- shards sharing a GPU encoded in
  // 287-316 ms what the default context does in 261 (r05final3), and varied from run to run
  if ((n_gpus == 1 || device_count() == 1) && !force_shards()) return mib_encode_batch(in, k, o, out, status);
  const int rc = run_shards(in, k, n_gpus, [&](Shard &sh, const std::vector<size_t> &idx) {
    return encode_shard(sh, in, idx, o, out, status);
  });
  if (rc)
    for (size_t i = 0; i < k; i++) mib_buf_free(&out[i]);
  return rc;
}

int mib_decode_batch_n(const mib_span *in, size_t k, int n_gpus, mib_buf *out, int *status) {
  if (k && (!in || !out || !status)) return MIB_E_INVALID_ARG;
  for (size_t i = 0; i < k; i++) {
    out[i].data = nullptr;
    out[i].size = 0;
    status[i] = 0;
    if (!in[i].data && in[i].size) return MIB_E_INVALID_ARG;
  }
  if (!k) return 0;
  if ((n_gpus == 1 || device_count() == 1) && !force_shards()) return mib_decode_batch(in, k, out, status);   // (as for the encode)
  const int rc = run_shards(
      in, k, n_gpus, [&](Shard &sh, const std::vector<size_t> &idx) { return decode_shard(sh, in, idx, out, status); },
      true);
  if (rc)
    for (size_t i = 0; i < k; i++) mib_buf_free(&out[i]);
  return rc;
}

int mib_device_count(void) { return device_count(); }

void mib_force_shards(int force) { __atomic_store_n(&g_force_shards, force ? 1 : 0, __ATOMIC_RELAXED); }

}  // extern "C"
