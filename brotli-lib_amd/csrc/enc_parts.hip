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
__global__ void ring_scan_kernel(Job *jobs, int njobs, Seg *segs, const PushSum *push) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= njobs) return;
  const Job &jb = jobs[j];
  if (jb.uncompressed) return;
  uint32_t ring[4];
  for (int q = 0; q < 4; q++) ring[q] = (uint32_t)jb.dc_in[q];
  for (uint32_t s = jb.seg_base; s < jb.seg_base + jb.nseg; s++) {
    for (int q = 0; q < 4; q++) segs[s].ring_in[q] = ring[q];
    const PushSum &ps = push[s];
    if (ps.n >= 4) {
      for (int q = 0; q < 4; q++) ring[q] = ps.d[q];
    } else if (ps.n) {
      uint32_t r[4];
      for (uint32_t q = 0; q < 4; q++) r[q] = q < ps.n ? ps.d[q] : ring[q - ps.n];
      for (int q = 0; q < 4; q++) ring[q] = r[q];
    }
  }
}
void launch_ring_scan(hipStream_t st, Job *jobs, int njobs, Seg *segs, int nsegs, const RawCmd *raw, PushSum *push) {
  hipLaunchKernelGGL(raw_push_kernel, dim3(nsegs), dim3(64), 0, st, jobs, segs, raw, push);
  hipLaunchKernelGGL(ring_scan_kernel, dim3((njobs + 63) / 64), dim3(64), 0, st, jobs, njobs, segs, push);
}

// Wave per stream: the entries in stream order, then the metadata block (window bits, header,
// payload) at the front of the stream's output slice.  The walk is serial in its state (ring,
// block types, remaining block lengths) but not in its inputs: the lanes stage 64 segments at
// a time (Seg, pushes, block-split units, the two bytes before the entry) in LDS, so the walk
// pays one memory round trip per 64 segments instead of several per segment.
constexpr int kPiChunk = 64;
__global__ __launch_bounds__(kPiChunk) void part_index_kernel(const Job *jobs, int njobs, const Mb *mbs, const Seg *segs,
                                                              const Unit *units, const PushSum *push, uint8_t *out) {
  __shared__ Seg s_seg[kPiChunk];
  __shared__ PushSum s_push[kPiChunk];
  __shared__ Unit s_unit[kPiChunk * kSubPerSeg];
  __shared__ uint32_t s_p12[kPiChunk];
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
  uint32_t ring[4];
  for (int q = 0; q < 4; q++) ring[q] = (uint32_t)jb.dc_in[q];
  const uint64_t bit0 = 8 * jb.out_base;
  const uint32_t seg_end = jb.seg_base + jb.nseg;
  uint32_t c0 = ~0u;   // first segment staged in LDS
  for (uint32_t m = 0; m < jb.nmb; m++) {
    const Mb &mb = mbs[jb.mb_base + m];
    uint32_t type[3] = {0, 0, 0}, prev[3] = {1, 1, 1}, blen[3];
    for (int c = 0; c < 3; c++) blen[c] = mb.nbt[c] > 1 ? mb.first_count[c] : (1u << 28);
    for (uint32_t s = mb.first_seg; s < mb.first_seg + mb.nseg; s++) {
      if (c0 == ~0u || s - c0 >= (uint32_t)kPiChunk) {   // (uniform) stage the next 64 segments
        c0 = s;
        __syncthreads();
        const uint32_t ls = c0 + lane;
        if (ls < seg_end) {
          const Seg sg = segs[ls];
          s_seg[lane] = sg;
          s_push[lane] = push[ls];
          const Mb &lm = mbs[sg.mb];
          const uint32_t p = ls == lm.first_seg ? lm.start : sg.start - sg.carry_in;
          s_p12[lane] = prev2(jb, p);
        }
        for (int i = lane; i < kPiChunk * kSubPerSeg; i += kPiChunk)
          if (c0 + i / kSubPerSeg < seg_end) s_unit[i] = units[(size_t)c0 * kSubPerSeg + i];
        __syncthreads();
      }
      const uint32_t k = s - c0;
      const Seg &sg = s_seg[k];
      const bool at_mb = s == mb.first_seg;
      if (lane == 0 && (s - jb.seg_base) % every == 0) {   // a part starts at this segment
        PartEntry e;
        const bool has_cmd = sg.ncmd + (sg.extra_ins ? 1 : 0) > 0;
        const uint32_t p = at_mb ? mb.start : sg.start - sg.carry_in;
        e.flags = at_mb ? (kPartValid | kPartAtMb) : has_cmd ? kPartValid : 0u;
        e.bit = bit0 + (at_mb ? mb.bit_off : sg.bit_off);
        e.pos = (uint64_t)jb.abs_base + p;
        e.mb_bit = bit0 + mb.bit_off;
        e.mb_pos = (uint64_t)jb.abs_base + mb.start;
        for (int q = 0; q < 4; q++) e.ring[q] = ring[q];
        for (int c = 0; c < 3; c++) {
          e.blen[c] = at_mb ? 0 : blen[c];
          e.type[c] = (uint8_t)(at_mb ? 0 : type[c]);
          e.prev[c] = (uint8_t)(at_mb ? 0 : prev[c]);
        }
        const uint32_t p12 = s_p12[k];
        e.p1 = (uint8_t)(p12 & 0xFF);
        e.p2 = (uint8_t)(p12 >> 8);
        const uint8_t *eb = reinterpret_cast<const uint8_t *>(&e);
        uint8_t *dst = ent + (size_t)((s - jb.seg_base) / every) * sizeof(PartEntry);
        for (int i = 0; i < (int)sizeof(e); i++) dst[i] = eb[i];
      }
      // the segment's distance pushes and block-split units, in stream order
      const PushSum &ps = s_push[k];
      if (ps.n >= 4) {
        for (int q = 0; q < 4; q++) ring[q] = ps.d[q];
      } else if (ps.n) {
        uint32_t r[4];
        for (uint32_t q = 0; q < 4; q++) r[q] = q < ps.n ? ps.d[q] : ring[q - ps.n];
        for (int q = 0; q < 4; q++) ring[q] = r[q];
      }
      for (int u = 0; u < kSubPerSeg; u++) {
        const Unit &un = s_unit[k * kSubPerSeg + u];
        for (int c = 0; c < 3; c++) {
          if (un.sw_count[c]) {
            prev[c] = type[c];
            type[c] = un.type[c];
            blen[c] = un.sw_count[c];
          }
          blen[c] -= un.nsym[c];
        }
      }
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
