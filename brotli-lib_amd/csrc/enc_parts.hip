// The part index (parts.h) of a stream: the decoder state at the first command of every
// 64 KiB parse segment, written as an RFC 7932 metadata metablock after the window bits.
// Everything it records is known once the commands are coded and the bit offsets are laid
// out: distance pushes per segment (part_push_kernel), then one walk per stream over its
// metablocks, segments and block-split units (part_index_kernel).
#include "enc_common.h"

namespace mib {
namespace enc {

struct PushSum {          // the explicit distances a segment pushes on the decoder's ring
  uint32_t n;             // how many
  uint32_t d[4];          // the last (up to) four, most recent first
};

// Wave per segment: walk the commands back to front 64 at a time; a command pushes its
// distance when it has a copy with an explicit distance code (code 0 = last distance and the
// implicit-distance commands do not push: engine.ts distance ring update).
__global__ __launch_bounds__(64) void part_push_kernel(const Job *jobs, const Seg *segs, const Cmd *cmds, PushSum *out) {
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const int lane = threadIdx.x;
  PushSum ps;
  ps.n = 0;
  for (int q = 0; q < 4; q++) ps.d[q] = 0;
  if (!jb.parts || jb.uncompressed) {
    if (lane == 0) out[blockIdx.x] = ps;
    return;
  }
  const Cmd *c = cmds + sg.cmd_off;
  const uint32_t n = sg.ncmd + (sg.extra_ins ? 1 : 0);
  uint32_t got = 0, total = 0;
  for (int64_t hi = (int64_t)n; hi > 0; hi -= 64) {
    const int64_t q = hi - 64 + lane;
    bool push = false;
    uint32_t d = 0;
    if (q >= 0) {
      const Cmd cc = c[q];
      push = cc.copy != 0 && (cc.dist_prefix & 0x3FF) != 0 && !is_word(jb, cc.dist);
      d = cc.dist;
    }
    uint64_t m = __ballot(push);
    total += (uint32_t)__popcll(m);
    while (m && got < 4) {
      const int l = 63 - __clzll((long long)m);
      ps.d[got++] = (uint32_t)__builtin_amdgcn_readlane((int)d, l);
      m &= ~(1ull << l);
    }
  }
  ps.n = total;
  if (lane == 0) out[blockIdx.x] = ps;
}

// The decoder's distance ring at every segment start (codes_kernel then picks short distance
// codes 1-15 from it, RFC 7932 section 4): the raw commands' pushes per segment -- a copy
// pushes its distance unless it equals the previous copy's (code 0) -- then a lane per stream
// walks its segments.  Every non-zero distance code pushes, so the ring does not depend on
// which of them a command ends up with.
__global__ __launch_bounds__(64) void raw_push_kernel(const Job *jobs, const Seg *segs, const RawCmd *raw, PushSum *out) {
  const Seg &sg = segs[blockIdx.x];
  const Job &jb = jobs[sg.job];
  const int lane = threadIdx.x;
  PushSum ps;
  ps.n = 0;
  for (int q = 0; q < 4; q++) ps.d[q] = 0;
  if (jb.uncompressed) {
    if (lane == 0) out[blockIdx.x] = ps;
    return;
  }
  const RawCmd *c = raw + sg.cmd_off;
  const int64_t n = sg.ncmd;
  uint32_t got = 0, total = 0;
  for (int64_t hi = n; hi > 0; hi -= 64) {
    const int64_t q = hi - 64 + lane;
    bool push = false;
    uint32_t d = 0;
    if (q >= 0) {
      d = c[q].dist;
      push = !is_word(jb, d) && d != (q ? c[q - 1].dist : sg.prev_dist);
    }
    uint64_t m = __ballot(push);
    total += (uint32_t)__popcll(m);
    while (m && got < 4) {
      const int l = 63 - __clzll((long long)m);
      ps.d[got++] = (uint32_t)__builtin_amdgcn_readlane((int)d, l);
      m &= ~(1ull << l);
    }
  }
  ps.n = total;
  if (lane == 0) out[blockIdx.x] = ps;
}
// Ring composition: the ring after pushes A then B (B's pushes are the more recent).
__device__ __forceinline__ PushSum push_then(const PushSum &a, const PushSum &b) {
  PushSum r;
  r.n = min(a.n + b.n, 1u << 30);
#pragma unroll
  for (uint32_t q = 0; q < 4; q++) r.d[q] = q < b.n ? b.d[q] : a.d[min(q - min(b.n, 4u), 3u)];
  return r;
}
__device__ __forceinline__ PushSum shfl_up_push(const PushSum &x, int o) {
  PushSum r;
  r.n = (uint32_t)__shfl_up((int)x.n, o);
#pragma unroll
  for (int q = 0; q < 4; q++) r.d[q] = (uint32_t)__shfl_up((int)x.d[q], o);
  return r;
}
// Wave-wide inclusive scan of the 64 lanes' push summaries (lane l: segments ..l composed)
__device__ __forceinline__ PushSum scan_pushes(PushSum x, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const PushSum y = shfl_up_push(x, o);
    if (lane >= o) x = push_then(y, x);
  }
  return x;
}
// the ring before a segment: the stream's incoming ring, then the pushes of the segments
// before it (an exclusive scan; ring as a PushSum with n >= 4)
__device__ __forceinline__ PushSum push_exclusive(const PushSum &carry, const PushSum &inc, int lane) {
  PushSum ex = shfl_up_push(inc, 1);
  if (lane == 0) ex.n = 0;
  return push_then(carry, ex);
}
// Wave per stream, 64 segments per step (a scan of their push summaries).
__global__ __launch_bounds__(64) void ring_scan_kernel(Job *jobs, int njobs, Seg *segs, const PushSum *push) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (j >= njobs) return;
  const Job &jb = jobs[j];
  if (jb.uncompressed) return;
  PushSum carry;
  carry.n = 4;
  for (int q = 0; q < 4; q++) carry.d[q] = (uint32_t)jb.dc_in[q];
  const uint32_t end = jb.seg_base + jb.nseg;
  for (uint32_t c0 = jb.seg_base; c0 < end; c0 += 64) {
    const uint32_t s = c0 + lane;
    PushSum x;
    x.n = 0;
    for (int q = 0; q < 4; q++) x.d[q] = 0;
    if (s < end) x = push[s];
    const PushSum inc = scan_pushes(x, lane);
    const PushSum before = push_exclusive(carry, inc, lane);
    if (s < end)
      for (int q = 0; q < 4; q++) segs[s].ring_in[q] = before.d[q];
    PushSum last;
    last.n = (uint32_t)__shfl((int)inc.n, 63);
    for (int q = 0; q < 4; q++) last.d[q] = (uint32_t)__shfl((int)inc.d[q], 63);
    carry = push_then(carry, last);
  }
}
void launch_ring_scan(hipStream_t st, Job *jobs, int njobs, Seg *segs, int nsegs, const RawCmd *raw, PushSum *push) {
  hipLaunchKernelGGL(raw_push_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, raw, push);
  hipLaunchKernelGGL(ring_scan_kernel, dim3(njobs), dim3(64), 0, st, jobs, njobs, segs, push);
}

// Block state of one category (type, previous type, remaining block length) as a composable
// summary of a run of segments: sw -- the run switches blocks (type, prev and blen are then
// the state after it; prev_in: prev is the type the run started with), else blen is the
// number of symbols the run consumes.  A metablock start is a switch to the header's state.
struct BlkSum {
  uint32_t blen;
  uint32_t sw, type, prev, prev_in;
};
__device__ __forceinline__ BlkSum blk_then(const BlkSum &a, const BlkSum &b) {
  if (!b.sw) {
    BlkSum r = a;
    r.blen = a.sw ? a.blen - b.blen : a.blen + b.blen;
    return r;
  }
  BlkSum r = b;
  if (b.prev_in && a.sw) {
    r.prev = a.type;
    r.prev_in = 0;
  }
  return r;
}
__device__ __forceinline__ BlkSum shfl_up_blk(const BlkSum &x, int o) {
  BlkSum r;
  r.blen = (uint32_t)__shfl_up((int)x.blen, o);
  r.sw = (uint32_t)__shfl_up((int)x.sw, o);
  r.type = (uint32_t)__shfl_up((int)x.type, o);
  r.prev = (uint32_t)__shfl_up((int)x.prev, o);
  r.prev_in = (uint32_t)__shfl_up((int)x.prev_in, o);
  return r;
}

// Wave per stream: the metadata block (window bits, header, payload) at the front of the
// stream's output slice, then the entries.  The state an entry records (ring, block types,
// remaining block lengths) is a prefix over the stream's segments: 64 segments per step, each
// lane summarises its segment (pushes; its block-split units, behind a reset where a
// metablock starts), a wave scan composes the summaries, and the lanes where a part starts
// write their entries.
constexpr int kPiChunk = 64;
__global__ __launch_bounds__(kPiChunk) void part_index_kernel(const Job *jobs, int njobs, const Mb *mbs, const Seg *segs,
                                                              const Unit *units, const PushSum *push, uint8_t *out) {
  const int j = blockIdx.x, lane = threadIdx.x;
  if (j >= njobs) return;
  const Job &jb = jobs[j];
  if (!jb.parts || jb.uncompressed) return;
  uint8_t *o = out + jb.out_off;
  const int wb = jb.hdr_lgwin ? window_bits_len((int)jb.hdr_lgwin) : 0;
  const int nb = part_skip_bytes(jb.idx_payload);
  const uint32_t every = 1u << (jb.part_bits - kSegBits);   // segments per part
  uint8_t *pay = o + ((uint64_t)(wb + 6 + 8 * nb) + 7) / 8;
  if (lane == 0) {
    BitW w{o, 0};
    if (jb.hdr_lgwin) put_window_bits(w, (int)jb.hdr_lgwin);
    w.put(1, 0);                       // ISLAST
    w.put(2, 3);                       // MNIBBLES: metadata
    w.put(1, 0);                       // reserved
    w.put(2, (uint32_t)nb);            // MSKIPBYTES
    w.put(8 * nb, jb.idx_payload - 1);   // MSKIPLEN - 1 (then zero bits to the byte boundary)
    PartHead h;
    h.magic = kPartMagic;
    h.version = 1;
    h.entry_bytes = (uint16_t)sizeof(PartEntry);
    h.nentries = (jb.nseg + every - 1) / every;
    h.lgwin = jb.lgwin;
    h.next_byte = jb.final_ ? 0 : jb.out_base + ((jb.total_bits + 7) >> 3);
    h.total = (uint64_t)jb.abs_base + jb.n;
    const uint8_t *hb = reinterpret_cast<const uint8_t *>(&h);
    for (int i = 0; i < (int)sizeof(h); i++) pay[i] = hb[i];
  }
  uint8_t *ent = pay + sizeof(PartHead);
  const uint64_t bit0 = 8 * jb.out_base;
  const uint32_t seg_end = jb.seg_base + jb.nseg;
  PushSum rcarry;   // the ring before the current 64 segments
  rcarry.n = 4;
  for (int q = 0; q < 4; q++) rcarry.d[q] = (uint32_t)jb.dc_in[q];
  BlkSum bcarry[3];   // the block state before them (the stream's first segment starts a metablock)
  for (int c = 0; c < 3; c++) bcarry[c] = BlkSum{0u, 1u, 0u, 1u, 0u};
  for (uint32_t c0 = jb.seg_base; c0 < seg_end; c0 += kPiChunk) {
    const uint32_t s = c0 + lane;
    const bool live = s < seg_end;
    PushSum ps;
    ps.n = 0;
    for (int q = 0; q < 4; q++) ps.d[q] = 0;
    BlkSum bs[3];
    for (int c = 0; c < 3; c++) bs[c] = BlkSum{0u, 0u, 0u, 0u, 0u};
    Seg sg{};
    bool at_mb = false;
    uint32_t mbi = 0;
    if (live) {
      sg = segs[s];
      ps = push[s];
      mbi = sg.mb;
      const Mb &mb = mbs[mbi];
      at_mb = s == mb.first_seg;
      if (at_mb)   // the metablock header's state: type 0, previous type 1, the first block's count
        for (int c = 0; c < 3; c++) bs[c] = BlkSum{mb.nbt[c] > 1 ? mb.first_count[c] : (1u << 28), 1u, 0u, 1u, 0u};
      for (int u = 0; u < kSubPerSeg; u++) {
        const Unit &un = units[(size_t)s * kSubPerSeg + u];
        for (int c = 0; c < 3; c++) {
          BlkSum &x = bs[c];
          if (un.sw_count[c]) {
            if (x.sw) {
              x.prev = x.type;
              x.prev_in = 0;
            } else {
              x.prev_in = 1;
            }
            x.sw = 1;
            x.type = un.type[c];
            x.blen = un.sw_count[c] - un.nsym[c];
          } else {
            x.blen = x.sw ? x.blen - un.nsym[c] : x.blen + un.nsym[c];
          }
        }
      }
    }
    // inclusive scans, then the state before each segment
    PushSum pinc = ps;
    BlkSum binc[3] = {bs[0], bs[1], bs[2]};
#pragma unroll
    for (int o = 1; o < kPiChunk; o <<= 1) {
      const PushSum py = shfl_up_push(pinc, o);
      if (lane >= o) pinc = push_then(py, pinc);
      for (int c = 0; c < 3; c++) {
        const BlkSum by = shfl_up_blk(binc[c], o);
        if (lane >= o) binc[c] = blk_then(by, binc[c]);
      }
    }
    const PushSum ring = push_exclusive(rcarry, pinc, lane);
    BlkSum before[3];
    for (int c = 0; c < 3; c++) {
      BlkSum ex = shfl_up_blk(binc[c], 1);
      if (lane == 0) ex = BlkSum{0u, 0u, 0u, 0u, 0u};
      before[c] = blk_then(bcarry[c], ex);
    }
    if (live && (s - jb.seg_base) % every == 0) {   // a part starts at this segment
      const Mb &mb = mbs[mbi];
      PartEntry e;
      const bool has_cmd = sg.ncmd + (sg.extra_ins ? 1 : 0) > 0;
      const uint32_t p = at_mb ? mb.start : sg.start - sg.carry_in;
      e.flags = at_mb ? (kPartValid | kPartAtMb) : has_cmd ? kPartValid : 0u;
      e.bit = bit0 + (at_mb ? mb.bit_off : sg.bit_off);
      e.pos = (uint64_t)jb.abs_base + p;
      e.mb_bit = bit0 + mb.bit_off;
      e.mb_pos = (uint64_t)jb.abs_base + mb.start;
      for (int q = 0; q < 4; q++) e.ring[q] = ring.d[q];
      for (int c = 0; c < 3; c++) {
        e.blen[c] = at_mb ? 0 : before[c].blen;
        e.type[c] = (uint8_t)(at_mb ? 0 : before[c].type);
        e.prev[c] = (uint8_t)(at_mb ? 0 : before[c].prev);
      }
      const uint32_t p12 = prev2(jb, p);
      e.p1 = (uint8_t)(p12 & 0xFF);
      e.p2 = (uint8_t)(p12 >> 8);
      const uint8_t *eb = reinterpret_cast<const uint8_t *>(&e);
      uint8_t *dst = ent + (size_t)((s - jb.seg_base) / every) * sizeof(PartEntry);
      for (int i = 0; i < (int)sizeof(e); i++) dst[i] = eb[i];
    }
    // carry the 64 segments' composition into the next step
    PushSum plast;
    plast.n = (uint32_t)__shfl((int)pinc.n, kPiChunk - 1);
    for (int q = 0; q < 4; q++) plast.d[q] = (uint32_t)__shfl((int)pinc.d[q], kPiChunk - 1);
    rcarry = push_then(rcarry, plast);
    for (int c = 0; c < 3; c++) {
      BlkSum bl;
      bl.blen = (uint32_t)__shfl((int)binc[c].blen, kPiChunk - 1);
      bl.sw = (uint32_t)__shfl((int)binc[c].sw, kPiChunk - 1);
      bl.type = (uint32_t)__shfl((int)binc[c].type, kPiChunk - 1);
      bl.prev = (uint32_t)__shfl((int)binc[c].prev, kPiChunk - 1);
      bl.prev_in = (uint32_t)__shfl((int)binc[c].prev_in, kPiChunk - 1);
      bcarry[c] = blk_then(bcarry[c], bl);
    }
  }
}

void launch_part_index(hipStream_t st, const Job *jobs, int njobs, const Mb *mbs, const Seg *segs, int nsegs,
                       const Cmd *cmds, const Unit *units, PushSum *push, uint8_t *out) {
  hipLaunchKernelGGL(part_push_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, cmds, push);
  hipLaunchKernelGGL(part_index_kernel, dim3(njobs), dim3(kPiChunk), 0, st, jobs, njobs, mbs, segs, units, push, out);
}

size_t part_push_bytes() { return sizeof(PushSum); }

}  // namespace enc
}  // namespace mib
