// brotli_amd: host batches sharded over several GPUs (SURVEY.md §8(b),(e): "batch calls are
// internally multi-GPU").  Independent buffers are assigned size-balanced to shards (the
// heaviest buffer to the least-loaded shard, like brotli_amd/shard.py), one host thread and
// one mib_ctx per shard; shard s runs on visible device s % device_count, so a one-GPU host
// can run two shards on one device (how the tests exercise the sharding).  Outputs come back
// in input order.  Only the public C ABI is used: each shard is an ordinary device-resident
// batch (mib_ctx_encode / mib_ctx_decode).  Nothing crosses between GPUs: the buffers are
// independent, so there is no collective; the results meet in host memory.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/brotli_amd.h"

// runtime.cpp: result buffers from device memory (mib_set_allocator's allocator)
extern "C" int mib_buf_from_device(mib_buf *out, const void *d_src, uint64_t len);
extern "C" int mib_bufs_from_device(size_t k, mib_buf *const *outs, const uint8_t *const *d_src, const uint64_t *len);

namespace {

constexpr int kMaxShards = 64;
std::mutex g_multi_mu;                 // one sharded call at a time: the shard contexts are reused
mib_ctx *g_shard_ctx[kMaxShards];      // shard s -> its context (device s % n), created on first use

int device_count() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
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

struct DevBuf {
  void *p = nullptr;
  ~DevBuf() {
    if (p) hipFree(p);
  }
  int alloc(uint64_t n) {
    return hipMalloc(&p, n ? n : 1) == hipSuccess ? 0 : MIB_E_OUT_OF_MEMORY;
  }
  uint8_t *u8() const { return (uint8_t *)p; }
};

int encode_shard(mib_ctx *c, const mib_span *in, const std::vector<size_t> &idx, const mib_enc_opts *o, mib_buf *out,
                 int *status) {
  const size_t k = idx.size();
  if (!k) return 0;
  std::vector<uint64_t> ioff(k + 1, 0), ooff(k + 1, 0);   // the shard's streams packed back to back
  uint64_t cap = 0;
  for (size_t q = 0; q < k; q++) {
    const uint64_t n = in[idx[q]].size;
    ioff[q + 1] = ioff[q] + n;
    cap += n + n / 8 + 8192 + ((n >> 16) + 1) * 72;   // (the encoder's bound: stored blocks + a part index)
  }
  DevBuf din, dout;
  int rc;
  if ((rc = din.alloc(ioff[k] + 64)) || (rc = dout.alloc(cap + 64))) return rc;
  for (size_t q = 0; q < k; q++)
    if (in[idx[q]].size && hipMemcpy(din.u8() + ioff[q], in[idx[q]].data, in[idx[q]].size, hipMemcpyHostToDevice) != hipSuccess)
      return MIB_E_NO_DEVICE;
  if ((rc = mib_ctx_encode(c, o, din.u8(), ioff.data(), k, dout.u8(), cap, ooff.data(), nullptr))) return rc;
  std::vector<mib_buf *> outs(k);
  std::vector<const uint8_t *> src(k);
  std::vector<uint64_t> lens(k);
  for (size_t q = 0; q < k; q++) {
    outs[q] = &out[idx[q]];
    src[q] = dout.u8() + ooff[q];
    lens[q] = ooff[q + 1] - ooff[q];
    status[idx[q]] = 0;
  }
  if ((rc = mib_bufs_from_device(k, outs.data(), src.data(), lens.data()))) return rc;
  return 0;
}

int decode_shard(mib_ctx *c, const mib_span *in, const std::vector<size_t> &idx, mib_buf *out, int *status) {
  const size_t k = idx.size();
  if (!k) return 0;
  std::vector<uint64_t> ioff(k + 1, 0), ooff(k + 1, 0);
  for (size_t q = 0; q < k; q++) {
    const mib_span &s = in[idx[q]];
    ioff[q + 1] = ioff[q] + s.size;
    const int64_t est = mib_decoded_size(s.data, s.size);
    // a header size, else room for a part-indexed stream's total (known only from its index),
    // else 8x the input; a stream that outgrows it is decoded again alone
    const uint64_t capq = est > 0 ? (uint64_t)est : std::max<uint64_t>(1 << 16, 8 * (uint64_t)s.size);
    ooff[q + 1] = ooff[q] + ((capq + 4096 + 255) & ~255ull);
  }
  DevBuf din, dout;
  int rc;
  if ((rc = din.alloc(ioff[k] + 64)) || (rc = dout.alloc(ooff[k] + 64))) return rc;
  for (size_t q = 0; q < k; q++)
    if (in[idx[q]].size && hipMemcpy(din.u8() + ioff[q], in[idx[q]].data, in[idx[q]].size, hipMemcpyHostToDevice) != hipSuccess)
      return MIB_E_NO_DEVICE;
  std::vector<int64_t> sizes(k);
  std::vector<int> st(k);
  rc = mib_ctx_decode(c, din.u8(), ioff.data(), k, dout.u8(), ooff.data(), sizes.data(), st.data(), nullptr);
  if (rc && rc != MIB_E_NEED_SPACE) return rc;
  for (size_t q = 0; q < k; q++) {
    const size_t i = idx[q];
    status[i] = st[q];
    if (st[q] == 0) {
      if ((rc = mib_buf_from_device(&out[i], dout.u8() + ooff[q], (uint64_t)sizes[q]))) return rc;
    } else if (st[q] == MIB_E_NEED_SPACE) {
      status[i] = mib_decode(in[i].data, in[i].size, nullptr, 0, -1, -1, &out[i]);   // the growing single-stream path
    }
  }
  return 0;
}

// run fn(shard, indices) on `shards` host threads; the first error wins
template <class F>
int run_shards(const mib_span *in, size_t k, int n_gpus, F fn) {
  const int ndev = device_count();
  if (ndev <= 0) return MIB_E_NO_DEVICE;
  int shards = n_gpus <= 0 ? ndev : n_gpus;
  shards = std::max(1, std::min<int>({shards, kMaxShards, (int)std::max<size_t>(k, 1)}));
  std::lock_guard<std::mutex> lk(g_multi_mu);
  for (int s = 0; s < shards; s++)
    if (!g_shard_ctx[s] && !(g_shard_ctx[s] = mib_ctx_new(s % ndev))) return MIB_E_NO_DEVICE;
  const std::vector<std::vector<size_t>> parts = assign(in, k, shards);
  std::vector<int> rcs(shards, 0);
  std::vector<std::thread> th;
  for (int s = 0; s < shards; s++)
    th.emplace_back([&, s] {
      hipSetDevice(s % ndev);
      rcs[s] = fn(g_shard_ctx[s], parts[s]);
    });
  for (auto &t : th) t.join();
  for (int r : rcs)
    if (r) return r;
  return 0;
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
  const int rc = run_shards(in, k, n_gpus, [&](mib_ctx *c, const std::vector<size_t> &idx) {
    return encode_shard(c, in, idx, o, out, status);
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
  const int rc = run_shards(in, k, n_gpus, [&](mib_ctx *c, const std::vector<size_t> &idx) {
    return decode_shard(c, in, idx, out, status);
  });
  if (rc)
    for (size_t i = 0; i < k; i++) mib_buf_free(&out[i]);
  return rc;
}

int mib_device_count(void) { return device_count(); }

}  // extern "C"
