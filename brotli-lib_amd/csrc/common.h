// Shared host/device definitions of the brotli_amd engine (job descriptors, status codes).
#pragma once
#include <stdint.h>

#include "../../include/brotli_amd.h"

// a result buffer (mib_buf.data) from the allocator mib_set_allocator chose (runtime.cpp)
extern "C" uint8_t *mib_buf_alloc(size_t n);
// out <- a new result buffer holding len bytes copied from device memory: 0 or MIB_E_*
extern "C" int mib_buf_from_device(mib_buf *out, const void *d_src, uint64_t len);
// *outs[i] <- len[i] bytes from d_src[i], i < k (one bulk copy when they are small)
extern "C" int mib_bufs_from_device(size_t k, mib_buf *const *outs, const uint8_t *const *d_src, const uint64_t *len);

namespace mib {

// Experiment knobs (MIB_* environment variables) are read only by the -DMIB_EXPERIMENTS build
// the A/B scripts make (`make EXPERIMENTS=1`, scripts/README.md).  The shipped library ignores
// the environment: its output depends on its inputs and options alone.
const char *knob(const char *name);

// Whether device `dev`'s returning LDS atomics served a wave's lanes in lane order in the
// self-test ensure_device runs once per device (mib_selftest_lds_atomic_order): the bucket
// sort's fast ranking relies on it, and ranks by ballots where it does not hold (enc_sort.hip).
bool lds_rank_ordered(int dev);

// Host <-> device copies of the host-buffer entry points through a context's pinned ring
// (runtime.cpp): upload returns once the host bytes are in the ring (copies queued on
// `stream`), download once every byte has reached host memory.
struct HostPiece {
  uint8_t *dst;
  const uint8_t *src;
  uint64_t n;
};
int ctx_upload(mib_ctx *c, void *stream, const HostPiece *ps, size_t k);
int ctx_download(mib_ctx *c, void *stream, const HostPiece *ps, size_t k);

// One stream to decode.  Filled by the host, read/written by decode kernels.
struct DecJob {
  const uint8_t *in;      // compressed stream (device)
  uint64_t in_len;
  uint8_t *out;           // output window (device), capacity out_cap (+64 B slack owned by us)
  uint64_t out_cap;
  int64_t out_size;       // > 0: known-size mode (brotliDecode pre-sizing / legacy outputSize)
  const uint8_t *dict;    // compound dictionary (device) or null
  uint64_t dict_len;
  int64_t result_len;     // out: bytes produced
  int32_t status;         // out: 0, reference error code, or MIB_E_*
  int32_t max_ring_log;   // window bits from the stream header (host peek), sizes scratch
  // part mode (parts.h): the job is one part of a stream that carries a part index
  const void *part_entry; // this part's PartEntry (device); null: a whole-stream job
  const void *next_entry; // the next part's entry, null for the stream's last part
  const int64_t *ppos;    // the stream's part start positions, [nparts] = its total
  uint64_t *prog;         // the stream's progress words (zeroed before the launch)
  int32_t pidx, nparts;
  int64_t total;          // the stream's decoded size (from the index)
};

constexpr int kDecodeBlock = 64;                    // one wave per stream
constexpr uint64_t kDecodeTableInts = 256u * (1 + 630) + 256u * (1 + 1080) + 256u * (1 + 1080) + 64;
constexpr uint64_t kDecodeCtxBytes = 256u * 64 + 256u * 4 + 256;

}  // namespace mib
