// Part index: decoder entry points that let one stream decode on many waves.
//
// A Brotli stream is one bit-serial chain, so a single stream decodes on one wave.  Streams
// produced by this encoder carry, in an RFC 7932 metadata metablock (skipped by every
// decoder, the reference's included: engine.ts ST_READ_METADATA), the decoder's complete
// state at the first command of every 64 KiB parse segment: bit position, output position,
// the metablock it is in, distance ring, block types and remaining block lengths, and the
// two context bytes.  A wave can then start at any entry (after decoding that entry's
// metablock header) and stop at the next one.  Copies reaching into an earlier part wait
// for that part's published progress; the encoder keeps such sources at offsets the
// earlier part has already decoded in lockstep (kPartLag below), so waits are rare.
//
// The parallel path is an optimisation with exact semantics: every part checks that its
// final state equals the next entry's, the last part must end the stream exactly as the
// serial decoder would, and any mismatch or error sends the stream through the serial
// decoder (which produces the reference's bytes and error codes).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MIB_HD __host__ __device__
#else
#define MIB_HD
#endif

namespace mib {

constexpr uint32_t kPartMagic = 0x3170424Du;     // "MBp1"
constexpr uint32_t kPartBits = 18;               // part size: 256 KiB (a multiple of the encoder's 64 KiB parse segment)
constexpr uint32_t kPartLag = 4096;              // an external copy source ends this far behind
                                                 // the destination's offset in its segment
#ifndef MIB_PART_PUBLISH
#define MIB_PART_PUBLISH 2048
#endif
constexpr uint32_t kPartPublish = MIB_PART_PUBLISH;   // a part publishes its progress this often (bytes)
constexpr uint64_t kPartMinStream = 2ull << 20;  // streams at least this long get a part index

constexpr uint32_t kPartValid = 1u;              // entry flags
constexpr uint32_t kPartAtMb = 2u;               // the entry is a metablock header

struct PartHead {          // 32 bytes, little endian, at the start of the metadata payload
  uint32_t magic;
  uint16_t version, entry_bytes;
  uint32_t nentries;
  uint32_t lgwin;
  uint64_t next_byte;      // stream byte offset of the next chunk's index block (0: none)
  uint64_t total;          // output bytes up to the end of this chunk
};

struct PartEntry {         // 72 bytes: the decoder state at a command boundary
  uint64_t bit;            // stream bit offset of the command (or of the metablock header)
  uint64_t pos;            // output position
  uint64_t mb_bit;         // bit offset of the header of the metablock holding pos
  uint64_t mb_pos;         // output position at which that metablock starts
  uint32_t ring[4];        // distance ring, most recent first
  uint32_t blen[3];        // remaining block lengths: literal, command, distance (0: switch next)
  uint8_t type[3], prev[3];   // current and previous block type per category
  uint8_t p1, p2;          // the two output bytes before pos
  uint32_t flags;
};
static_assert(sizeof(PartHead) == 32, "part head layout");
static_assert(sizeof(PartEntry) == 72, "part entry layout");

// metadata metablock framing of a payload of n bytes at bit offset b (after the window bits):
// ISLAST 0, MNIBBLES 0 (code 3), reserved 0, MSKIPBYTES, MSKIPLEN - 1, pad to a byte
MIB_HD inline int part_skip_bytes(uint64_t n) { return n <= 256 ? 1 : n <= 65536 ? 2 : 3; }
MIB_HD inline uint64_t part_index_bits(int wbits, uint64_t payload) {
  const uint64_t hdr = (uint64_t)wbits + 6 + 8 * (uint64_t)part_skip_bytes(payload);
  return ((hdr + 7) & ~7ull) + 8 * payload;
}
MIB_HD inline int window_bits_len(int lg) { return lg == 16 ? 1 : lg > 17 ? 4 : 7; }

}  // namespace mib
