// kern_b64.hpp -- the receiver's base64 decode on the device (gfx950).
//
// A SendChunk frame carries the chunk as XML-RPC base64 text
// (/root/reference/cpp/src/ChunkMethods.cpp:141-163, decoded by xmlrpc++ 0.7
// XmlRpcValue::binaryFromXml, XmlRpcValue.cpp:417-436, with the decoder of
// base64.h:215-330).  lbf_b64_verify_batch decodes each chunk's text here, in
// HBM, and the shipped hash kernels verify the decoded bytes where they lie,
// so the receiver's two per-chunk passes (decode, then hash) both run on the
// GPU and only the text crosses PCIe on the way in.
//
// Decode rules (base64.h:215-330, restated in bitflood_amd/host/PeerWire.cpp
// Base64Get and tests/test_gpu_b64.py):
//   - characters outside the alphabet (the frame's spaces, anything else) are
//     skipped;
//   - the remaining characters S[0..m) are taken four at a time; a group that
//     holds '=' ends the data: "xx==" gives one byte, "xxx=" two, '=' in the
//     first or second place none; an incomplete last group gives nothing.
// So with q = the index of the first '=' in S (m if none), the output is the
// 3 * floor(min(q, m) / 4) bytes of the complete groups, plus one byte when
// q % 4 == 2 or two when q % 4 == 3 (q < m).
//
// Text laid out as the encoder writes it (nearly every frame) goes through
// b64_decode_canon_kernel: one pass, each lane decodes four groups from their
// known places, 7/3 bytes moved per decoded byte.  Any other text goes through
// b64_decode_kernel, one workgroup per chunk: pass 1 compacts the text (4 KiB
// tiles, each lane classifies 16 characters, a workgroup scan gives every
// valid character its index in S, and the sextets are written to a scratch
// area laid out like the text); pass 2 turns four groups (16 sextets, one
// 16-byte load) into 12 bytes per lane.  5 bytes moved per decoded byte (4/3
// each for the text read and the sextets written and read back, 1 for the
// bytes written).
//
// Part of the single translation unit sha1_kernels.hip (included from there).
#pragma once

#include <hip/hip_runtime.h>

#include "lbf_internal.hpp"

namespace lbf {
namespace {

constexpr uint8_t kB64Eq = 64, kB64Skip = 255;
constexpr int kB64Threads = 256;  // one lane per entry of the decode table below

struct B64Table {
  uint8_t v[256];
};

constexpr B64Table make_b64_table() {
  B64Table t{};
  for (int c = 0; c < 256; ++c) t.v[c] = kB64Skip;
  for (int c = 'A'; c <= 'Z'; ++c) t.v[c] = (uint8_t)(c - 'A');
  for (int c = 'a'; c <= 'z'; ++c) t.v[c] = (uint8_t)(26 + c - 'a');
  for (int c = '0'; c <= '9'; ++c) t.v[c] = (uint8_t)(52 + c - '0');
  t.v['+'] = 62;
  t.v['/'] = 63;
  t.v['='] = kB64Eq;
  return t;
}

__constant__ B64Table g_b64_table = make_b64_table();

// Exclusive scan of one value per lane over the 256-lane workgroup; returns
// the lane's prefix and writes the total to *total.  `sums` is 4 words of LDS.
__device__ __forceinline__ uint32_t wg_exclusive_scan(uint32_t v, uint32_t* sums, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sums[wave] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kB64Threads / 64; ++w) {
    const uint32_t s = sums[w];
    before += w < wave ? s : 0u;
    all += s;
  }
  __syncthreads();  // sums is reused by the next call
  *total = all;
  return before + x - v;
}

// ---------------------------------------------------------------------------
// Tiles of whole lines.  The encoder's text is lines of 18 groups: 72 alphabet
// characters and a separator (base64.h:197-205's '\n', framed as a space), 73
// characters that decode to 54 bytes.  A tile of L lines is 73L characters
// and 54L bytes, so tile k of a chunk reads text [73Lk, +73L) and writes bytes
// [54Lk, +54L) (or the reverse for the encode), and no group or separator
// crosses a tile; where the tile's output is whole 16-byte blocks it is
// written with 16-byte stores whenever the chunk's slot is 16-byte aligned.
// grid = (groups of tiles, chunks); every workgroup stages its tile's input
// span in LDS with coalesced 16-byte loads (global_load_dwordx4 +
// ds_write_b128), then each lane builds one or two 16-byte blocks of the output
// from LDS and stores them: one pass over HBM in each direction, nothing
// re-read.  (Round 4's kernels read bytes straight from HBM,
// 16 byte loads per four groups per lane, and spent 74-86 % of their wave
// cycles waiting on memory at 0.23-0.30 of the HBM peak)
// ---------------------------------------------------------------------------
// The encode's tile: 112 lines, 6,048 bytes -> 8,176 characters = 511 output
// blocks, two per lane (64 lines made 292 blocks: a second pass for 36 lanes).
// 120.5-121.0 us per 1,024 x 256 KiB against 136.1-137.4 for 64 lines, alternating on one box
// (profiles/r05/b64_geometry/ab_traces_enc_tiles.json).  Both texts and bytes of
// a tile must be whole 16-byte blocks: a multiple of 16 lines.
#ifndef LBF_B64_ENC_LINES
#define LBF_B64_ENC_LINES 112
#endif
constexpr uint32_t kB64TileLines = LBF_B64_ENC_LINES;
constexpr uint32_t kB64TileText = kB64TileLines * 73;    // 8,176 characters
constexpr uint32_t kB64TileBytes = kB64TileLines * 54;   // 6,048 bytes
constexpr uint32_t kB64TileGroups = kB64TileLines * 18;  // 2,016 groups
static_assert(kB64TileText % 16 == 0 && kB64TileBytes % 16 == 0, "tiles of 16-byte blocks");
// The decode's tile (its output, the bytes, must be whole 16-byte blocks: a
// multiple of 8 lines; its text tile is read at any phase): 72 lines, 5,256
// characters -> 3,888 bytes, 243 of the 256 lanes busy (64 lines: 216).  That
// and eight tiles per workgroup measured 157.6 us per 1,024 x 256 KiB against
// 171.5-171.8 for 64 lines and four (tools/b64_ab_trace.sh, profiles/r05/b64/);
// 144 lines (two blocks per lane) measured 175-179 us.  The leaner block below
// (62 VGPRs, 8 waves per SIMD) then runs best at four tiles per workgroup:
// 129.7-130.7 us (profiles/r05/b64_geometry/ab_traces_dec_v2.json).
// LBF_B64_DEC_LINES, LBF_B64_DEC_TILES_PER_GROUP and LBF_B64_ENC_TILES_PER_GROUP
// exist for A/B builds (tools/b64_ab_build.sh).
#ifndef LBF_B64_DEC_LINES
#define LBF_B64_DEC_LINES 72
#endif
#ifndef LBF_B64_DEC_WIN64
#define LBF_B64_DEC_WIN64 0
#endif
constexpr uint32_t kDecLines = LBF_B64_DEC_LINES;
constexpr uint32_t kDecText = kDecLines * 73, kDecBytes = kDecLines * 54, kDecGroups = kDecLines * 18;
static_assert(kDecBytes % 16 == 0, "a decode tile is whole 16-byte blocks of output");
typedef uint32_t b64_u32x4 __attribute__((ext_vector_type(4)));  // what the nontemporal builtins take

// Stage global bytes [src, src + len) in LDS as the aligned 16-byte blocks that
// hold them: afterwards lds byte (delta + k) = src[k], delta = src mod 16.  The
// blocks are read whole (a 16-byte block holding one byte of the span lies in
// the same page, so this never reads an unmapped address).  Up to kPer blocks
// per lane.  load() issues all of a lane's loads and returns at once; store()
// waits for them and writes LDS, so work placed between the two (the decode
// table, the last group's check) runs while the loads are in flight.
template <uint32_t kPer>
struct B64Stage {
  b64_u32x4 v[kPer];
  uint32_t blocks = 0, delta = 0;
  __device__ __forceinline__ void load(const uint8_t* src, uint32_t len) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(src);
    delta = (uint32_t)(a & 15u);
    const b64_u32x4* g = reinterpret_cast<const b64_u32x4*>(a - delta);
    blocks = (delta + len + 15) / 16;
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      if (threadIdx.x + k * kB64Threads < blocks) v[k] = __builtin_nontemporal_load(g + threadIdx.x + k * kB64Threads);
  }
  __device__ __forceinline__ void store(uint4* lds) const {
    b64_u32x4* l = reinterpret_cast<b64_u32x4*>(lds);
#pragma unroll
    for (uint32_t k = 0; k < kPer; ++k)
      if (threadIdx.x + k * kB64Threads < blocks) l[threadIdx.x + k * kB64Threads] = v[k];
  }
};

// The decode table entry of character c (B64Table), computed: filling the LDS
// copy this way costs a few VALU per lane and no dependent global load.
__device__ __forceinline__ uint32_t b64_value(uint32_t c) {
  return c - 'A' < 26u ? c - 'A' : c - 'a' < 26u ? c - 'a' + 26 : c - '0' < 10u ? c - '0' + 52 :
         c == '+' ? 62u : c == '/' ? 63u : c == '=' ? (uint32_t)kB64Eq : (uint32_t)kB64Skip;
}

// Four bytes of LDS from any byte address (two aligned dword reads + v_alignbyte).
__device__ __forceinline__ uint32_t lds_u32_at(const uint32_t* w, uint32_t at) {
  return __builtin_amdgcn_alignbyte(w[(at >> 2) + 1], w[at >> 2], at & 3u);
}

// Store a 16-byte block to dst = base + pos, clipped to [0, end) of the slot:
// one 16-byte store when it is whole and aligned, bytes otherwise.
__device__ __forceinline__ void b64_put_block(uint8_t* base, uint64_t pos, uint64_t end, uint4 v) {
  uint8_t* dst = base + pos;
  if (pos + 16 <= end && (reinterpret_cast<uintptr_t>(dst) & 15u) == 0) {
    const b64_u32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<b64_u32x4*>(dst));
    return;
  }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t m = 0; m < 16 && pos + m < end; ++m) dst[m] = (uint8_t)(w[m >> 2] >> (8 * (m & 3)));
}

// ---------------------------------------------------------------------------
// One pass for text laid out as the encoder writes it (round 4; tiled in
// round 5).  Almost every frame carries exactly what xmlrpc++'s encoder
// wrote: group g of the chunk at 4g + g/18, a separator (any character outside
// the alphabet) after every 18th group, '=' only as "xx==" / "xxx=" in the
// last group.  For such a text the place of every character is known without
// a scan.  The lanes check the layout as they read it; a chunk whose text
// breaks it anywhere (junk, a dropped or extra character, '=' elsewhere) is
// marked in redo[] and decoded again by b64_decode_kernel, whose general rules
// give the same result as this pass on every canonical text.
//
// The length gives the group count.  The encoder writes a separator after
// every 18th complete group, so a text of G = 18q + r groups (0 < r < 18 or
// r = 0) has length 73q + 4r, and one whose last, padded group is the 18th of
// its line has no separator after it: 73q + 72, G = 18(q + 1).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool b64_canon_groups(uint32_t len, uint32_t* groups) {
  const uint32_t q = len / 73, rem = len % 73;
  if (rem == 72) {  // the last line's 18th group is the padded last group
    *groups = 18 * q + 18;
    return true;
  }
  if (rem % 4 != 0) return false;
  *groups = 18 * q + rem / 4;
  return true;
}

// One block of a tile of the one-pass decode from its text in LDS (sb, from
// byte `delta`): in pass p, lane v builds and stores bytes [16u, 16u + 16) of
// the tile, u = v + 256p (if the tile has that block).  Returns true when the
// lane saw a character that breaks the layout.  The kernel is VALU-bound
// (about 70 % of its time was VALU issue at 230 instructions per block), so the
// block keeps its instruction count down: the layout checks fold into two flag
// words, the sextets are joined unmasked, and the 18 bytes are packed with five
// v_perm_b32 (157 -> 133 us per 1,024 x 256 KiB).
template <uint32_t kPass>
__device__ __forceinline__ bool b64_decode_block(const uint8_t* sb, uint32_t delta, const uint8_t* tab, uint32_t tile,
                                                 uint32_t groups, uint32_t len, uint64_t want, uint32_t limit,
                                                 uint8_t* o) {
  if (threadIdx.x + kPass * kB64Threads >= kDecBytes / 16) return false;
  // Bytes [16u, 16u + 16) of the tile come from its groups g0 .. g0 + 5, whose
  // characters lie in [c0, c0 + 25): 24 characters and at most one separator,
  // after group 17 - r0 of the window when r0 >= 12.  One window of eight
  // aligned dwords holds them; each group's four characters are cut out of it
  // with v_alignbyte (no divergent branch: groups past the chunk's end are
  // decoded from whatever lies there and masked below).
  const uint32_t* w = reinterpret_cast<const uint32_t*>(sb);
  const uint32_t b0 = 16 * (threadIdx.x + kPass * kB64Threads), g0 = b0 / 3, phase = b0 - 3 * g0;
  const uint32_t l0 = g0 / 18, r0 = g0 - 18 * l0;
  const uint32_t c0 = delta + 4 * g0 + l0, sh0 = c0 & 3u;
#if LBF_B64_DEC_WIN64
  // A/B: the window as five 8-byte reads from the even dword below it.  Lanes'
  // windows start ~5.3 dwords apart, so eight ds_read_b32 (banks (a/4) mod 32,
  // 32-lane groups) meet ~3-way bank conflicts; ds_read_b64 banks mod 64.
  const uint32_t r = (c0 >> 2) & 1u;
  const uint2* wb = reinterpret_cast<const uint2*>(w + ((c0 >> 2) & ~1u));
  uint32_t win[10];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint2 x2 = wb[k];
    win[2 * k] = x2.x;
    win[2 * k + 1] = x2.y;
  }
#else
  const uint32_t* wb = w + (c0 >> 2);
  uint32_t win[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) win[k] = wb[k];
#endif
  const uint32_t gbase = tile * kDecGroups + g0;  // the chunk's index of group g0
  bool bad = false;
  uint32_t x[6];
  // Table entries are 0..63, '=' 64 and anything else 255, so (entry >> 6)
  // is 0 exactly for an alphabet character: two flag bits per group, at 2j,
  // for all four characters (finner) and the first two (fhead).
  uint32_t finner = 0, fhead = 0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const uint32_t sep = r0 + j >= 18 ? 1u : 0u;
    const uint32_t off = sh0 + sep;  // 0..4: this group's offset from dword j of the window
#if LBF_B64_DEC_WIN64
    const uint32_t q = r + (off >> 2);  // 0..2 dwords past win[j]
    const uint32_t lo = q == 0 ? win[j] : q == 1 ? win[j + 1] : win[j + 2];
    const uint32_t hi = q == 0 ? win[j + 1] : q == 1 ? win[j + 2] : win[j + 3];
#else
    const uint32_t lo = off >= 4 ? win[j + 1] : win[j], hi = off >= 4 ? win[j + 2] : win[j + 1];
#endif
    const uint32_t c = __builtin_amdgcn_alignbyte(hi, lo, off & 3u);
    const uint32_t s0 = tab[c & 255], s1 = tab[(c >> 8) & 255], s2 = tab[(c >> 16) & 255], s3 = tab[c >> 24];
    const uint32_t o2 = s0 | s1, o4 = o2 | s2 | s3;
    finner |= (o4 >> 6) << (2 * j);
    fhead |= (o2 >> 6) << (2 * j);
    // unmasked: an entry above 63 spoils only its own group's bytes, and such a
    // group is either marked bad or the last group's '=' padding, whose bytes
    // (those a '=' in character 2 or 3 reaches) lie past the decoded length
    // and are zeroed below
    x[j] = (((s0 << 6) | s1) << 12) | ((s2 << 6) | s3);
  }
  {
    // window groups j < rel lie inside the text (all four characters in the
    // alphabet); group rel is the chunk's last (its first two in the alphabet;
    // the kernel checks its padding)
    const int32_t rel = (int32_t)groups - 1 - (int32_t)gbase;
    const uint32_t nin = (uint32_t)min(max(rel, 0), 6);
    const uint32_t inner_mask = (1u << (2 * nin)) - 1u;
    const uint32_t head_mask = rel >= 0 && rel < 6 ? 3u << (2 * rel) : 0u;
    bad |= ((finner & inner_mask) | (fhead & head_mask)) != 0;
  }
  // the separator after group 17 - r0 (when in the window): any character outside the alphabet
  {
    const uint32_t js = 17 - r0;  // < 6 when r0 >= 12
    const uint32_t gs = gbase + js;
    const uint32_t at = (c0 & ~3u) + min(sh0 + 4 * js + 4, 31u);
    const bool check = r0 >= 12 && 4 * gs + gs / 18 + 4 < len;
    bad |= check && tab[sb[at]] != kB64Skip;
  }
  // the 18 bytes of the six groups, as little-endian words
  // group j's bytes are x[j]'s bytes 2, 1, 0: one v_perm_b32 per word (selector
  // bytes 0-3 pick from the second source, 4-7 from the first, 12 gives 0)
  const uint32_t W0 = __builtin_amdgcn_perm(x[1], x[0], 0x06000102u);
  const uint32_t W1 = __builtin_amdgcn_perm(x[2], x[1], 0x05060001u);
  const uint32_t W2 = __builtin_amdgcn_perm(x[3], x[2], 0x04050600u);
  const uint32_t W3 = __builtin_amdgcn_perm(x[5], x[4], 0x06000102u);
  const uint32_t W4 = __builtin_amdgcn_perm(x[5], x[5], 0x0C0C0001u);
  uint4 v = make_uint4(__builtin_amdgcn_alignbyte(W1, W0, phase), __builtin_amdgcn_alignbyte(W2, W1, phase),
                       __builtin_amdgcn_alignbyte(W3, W2, phase), __builtin_amdgcn_alignbyte(W4, W3, phase));
  const uint64_t pos = (uint64_t)tile * kDecBytes + b0;
  if (pos < limit) {
    if (pos + 16 > want) {  // the decoded bytes end inside this block: zero the rest of the slot
      uint32_t ws[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int m = 0; m < 16; ++m)
        if (pos + m >= want) ws[m >> 2] &= ~(255u << (8 * (m & 3)));
      v = make_uint4(ws[0], ws[1], ws[2], ws[3]);
    }
    b64_put_block(o, pos, limit, v);
  }
  return bad;
}

// A tile: every lane its block of each pass (one pass for the shipped 243-block
// tile; the block index is written out in each pass rather than passed in, which
// kept the shipped kernel at 71 VGPRs where a block-index argument made it 87).
__device__ __forceinline__ bool b64_decode_tile(const uint8_t* sb, uint32_t delta, const uint8_t* tab, uint32_t tile,
                                                uint32_t groups, uint32_t len, uint64_t want, uint32_t limit,
                                                uint8_t* o) {
  static_assert(kDecBytes / 16 <= 3 * kB64Threads, "three blocks per lane at most");
  bool bad = b64_decode_block<0>(sb, delta, tab, tile, groups, len, want, limit, o);
  if constexpr (kDecBytes / 16 > kB64Threads) bad |= b64_decode_block<1>(sb, delta, tab, tile, groups, len, want, limit, o);
  if constexpr (kDecBytes / 16 > 2 * kB64Threads)
    bad |= b64_decode_block<2>(sb, delta, tab, tile, groups, len, want, limit, o);
  return bad;
}

// Tiles per workgroup: a workgroup takes kDecTilesPerGroup (kEncTilesPerGroup) consecutive tiles
// of its chunk and double-buffers them in LDS, so the next tile's loads are in
// flight while it decodes (or encodes) the current one: one barrier per tile,
// and a CU's resident workgroups keep loads outstanding through their compute.
#ifndef LBF_B64_DEC_TILES_PER_GROUP
#define LBF_B64_DEC_TILES_PER_GROUP 4  // 2, 3, 6, 8: 141, 134, 140, 133 us against 130 (256 KiB chunks: 68 tiles)
#endif
#ifndef LBF_B64_ENC_TILES_PER_GROUP
#define LBF_B64_ENC_TILES_PER_GROUP 2  // of 112 lines (1 and 3: 0.5-1 % slower; 64-line tiles: 4, eight 5 % slower)
#endif
constexpr uint32_t kDecTilesPerGroup = LBF_B64_DEC_TILES_PER_GROUP, kEncTilesPerGroup = LBF_B64_ENC_TILES_PER_GROUP;

// blockIdx.x = group of tiles, blockIdx.y = chunk - chunk0.  Chunk i's text is
// text[text_off[i] .. + text_len[i]); its decoded bytes go to
// out[out_off[i] .. + cap[i]): bytes [0, min(decoded, cap)) decoded, the rest
// of the slot zeroed, so a short text never leaves stale device bytes in the
// caller's slot.  sizes[i] = min(decoded, cap[i]), over[i] = decoded > cap[i].
// `tiles` = the tiles that cover the chunk with the most (text or slot).
__global__ void __launch_bounds__(kB64Threads) b64_decode_canon_kernel(const uint8_t* __restrict__ text,
                                                                       const uint64_t* __restrict__ text_off,
                                                                       const uint32_t* __restrict__ text_len,
                                                                       uint8_t* __restrict__ out,
                                                                       const uint64_t* __restrict__ out_off,
                                                                       const uint32_t* __restrict__ cap,
                                                                       uint32_t* __restrict__ sizes,
                                                                       uint8_t* __restrict__ over,
                                                                       uint8_t* __restrict__ redo, uint32_t tiles,
                                                                       uint32_t chunk0) {
  // a tile's span, its phase, and slack for the last lane's 32-byte window read
  constexpr uint32_t kStage = (kDecText + 15 + 15) / 16 + 2;
  constexpr uint32_t kPer = (kStage + kB64Threads - 1) / kB64Threads;  // staged blocks per lane
  __shared__ uint4 stage[2][kStage];
  __shared__ uint8_t tab[256];
  __shared__ uint32_t last_shared;
  const uint32_t i = chunk0 + blockIdx.y, t0 = blockIdx.x * kDecTilesPerGroup;
  const uint32_t len = text_len[i];
  uint32_t groups = 0;
  if (!b64_canon_groups(len, &groups)) {  // the whole workgroup leaves: no barrier below is reached
    if (t0 == 0 && threadIdx.x == 0) redo[i] = 1;
    return;
  }
  const uint32_t limit = cap[i];
  // the tiles this chunk has: its text's and its slot's (at least one, for the sizes)
  const uint32_t own = max(1u, max((len + kDecText - 1) / kDecText,
                                   (limit + kDecBytes - 1) / kDecBytes));
  if (t0 >= own) return;  // the whole workgroup
  const uint32_t t1 = min(own, t0 + kDecTilesPerGroup);
  const uint8_t* t = text + text_off[i];
  uint8_t* o = out + out_off[i];
  B64Stage<kPer> st;
  auto load = [&](uint32_t tile) {
    const uint32_t tbeg = tile * kDecText;
    st.blocks = 0;
    st.delta = 0;
    if (tbeg < len) st.load(t + tbeg, min(kDecText, len - tbeg));
  };
  load(t0);
  tab[threadIdx.x] = (uint8_t)b64_value(threadIdx.x);
  if (threadIdx.x == 0) {
    // the last group -- "xxxx", "xxx=" or "xx==" -- sets the decoded length
    uint32_t last = 3;
    bool bad = false;
    if (groups > 0) {
      const uint32_t g = groups - 1, at = 4 * g + g / 18;
      const uint32_t c2 = b64_value(t[at + 2]), c3 = b64_value(t[at + 3]);
      last = c3 < 64 ? 3u : c2 < 64 ? 2u : 1u;
      bad = c3 == kB64Skip || c2 == kB64Skip || (c2 == kB64Eq && c3 != kB64Eq);
    }
    last_shared = last;
    if (t0 == 0) {
      const uint64_t want = groups ? 3ull * (groups - 1) + last : 0;
      sizes[i] = (uint32_t)min<uint64_t>(want, limit);
      over[i] = want > limit ? 1 : 0;
      if (bad) redo[i] = 1;
    }
  }
  st.store(stage[0]);
  uint32_t delta = st.delta;
  __syncthreads();
  const uint64_t want = groups ? 3ull * (groups - 1) + last_shared : 0;
  bool bad = false;
  for (uint32_t tile = t0; tile < t1; ++tile) {
    const uint32_t buf = (tile - t0) & 1u;
    if (tile + 1 < t1) load(tile + 1);  // in flight while this tile decodes
    bad |= b64_decode_tile(reinterpret_cast<const uint8_t*>(stage[buf]), delta, tab, tile, groups, len, want, limit, o);
    if (tile + 1 < t1) {
      st.store(stage[buf ^ 1u]);  // that buffer's last reader was the previous tile, before the last barrier
      delta = st.delta;
      __syncthreads();
    }
  }
  if (bad) redo[i] = 1;  // every writer stores the same 1
}

// blockIdx.x = chunk (skipped when redo is given and redo[chunk] == 0).
// Chunk i's text is text[text_off[i] .. + text_len[i])
// (any alignment; 4-byte aligned reads faster) and its sextets go to
// scratch[sext_off[i] ..) (16-byte aligned, room for text_len[i]: the
// compacted stream is never longer than the text).  out[out_off[i] .. + cap[i])
// receives the decoded bytes; sizes[i] = min(decoded length, cap[i]) and
// over[i] = 1 when the text decodes to more than cap[i] bytes.
__global__ void __launch_bounds__(kB64Threads) b64_decode_kernel(const uint8_t* __restrict__ text,
                                                                 uint8_t* __restrict__ scratch,
                                                                 const uint64_t* __restrict__ text_off,
                                                                 const uint64_t* __restrict__ sext_off,
                                                                 const uint32_t* __restrict__ text_len,
                                                                 uint8_t* __restrict__ out,
                                                                 const uint64_t* __restrict__ out_off,
                                                                 const uint32_t* __restrict__ cap,
                                                                 uint32_t* __restrict__ sizes,
                                                                 uint8_t* __restrict__ over,
                                                                 const uint8_t* __restrict__ redo) {
  // after b64_decode_canon_kernel: only the chunks it could not take
  if (redo && !redo[blockIdx.x]) return;
  __shared__ uint32_t sums[kB64Threads / 64];
  __shared__ uint32_t first_eq;
  __shared__ uint8_t tab[256];  // per-lane lookups: LDS serves divergent addresses, the constant table does not
  tab[threadIdx.x] = g_b64_table.v[threadIdx.x];
  const uint32_t i = blockIdx.x;
  const uint8_t* t = text + text_off[i];
  uint8_t* s = scratch + sext_off[i];
  const uint32_t len = text_len[i];
  if (threadIdx.x == 0) first_eq = 0xFFFFFFFFu;
  __syncthreads();
  // ---- pass 1: compact the alphabet characters (and '=') into sextets ----
  uint32_t base = 0;  // sextets written by earlier tiles
  for (uint32_t tile = 0; tile < len; tile += kB64Threads * 16) {
    const uint32_t at = tile + threadIdx.x * 16;
    uint8_t c[16];
    if (at + 16 <= len) {
      // the text of a chunk need not be 16-byte aligned: four dword loads
      // when it is 4-byte aligned, bytes otherwise
      if ((reinterpret_cast<uintptr_t>(t + at) & 3u) == 0) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(t + at);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t w = p[k];
          c[4 * k] = (uint8_t)w;
          c[4 * k + 1] = (uint8_t)(w >> 8);
          c[4 * k + 2] = (uint8_t)(w >> 16);
          c[4 * k + 3] = (uint8_t)(w >> 24);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) c[k] = t[at + k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) c[k] = at + k < len ? t[at + k] : (uint8_t)' ';
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      c[k] = tab[c[k]];
      cnt += c[k] != kB64Skip;
    }
    uint32_t total;
    uint32_t pos = base + wg_exclusive_scan(cnt, sums, &total);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (c[k] == kB64Skip) continue;
      if (c[k] == kB64Eq) atomicMin(&first_eq, pos);
      s[pos++] = c[k];
    }
    base += total;
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t m = base, q = min(first_eq, m);
  const uint32_t groups = q / 4;  // complete groups before any '='
  const uint32_t r = q % 4;
  // q < m: S[q] is '=': "xx=" gives one byte, "xxx=" two.  q == m: an
  // incomplete last group gives nothing.
  const uint32_t extra = q < m ? (r == 2 ? 1u : r == 3 ? 2u : 0u) : 0u;
  const uint64_t want = 3ull * groups + extra;
  const uint32_t limit = cap[i];
  uint8_t* o = out + out_off[i];
  // ---- pass 2: four groups (16 sextets) -> 12 bytes per lane ----
  for (uint32_t g4 = threadIdx.x * 4; g4 < groups; g4 += kB64Threads * 4) {
    uint8_t v[16];
    if (g4 + 4 <= groups) {
      const uint4 w = *reinterpret_cast<const uint4*>(s + 4ull * g4);  // 16-byte aligned: s is
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = (uint8_t)(ws[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = 4 * g4 + k < 4ull * groups ? s[4 * g4 + k] : (uint8_t)0;
    }
    uint8_t b[12];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = ((uint32_t)v[4 * k] << 18) | ((uint32_t)v[4 * k + 1] << 12) | ((uint32_t)v[4 * k + 2] << 6) |
                         v[4 * k + 3];
      b[3 * k] = (uint8_t)(x >> 16);
      b[3 * k + 1] = (uint8_t)(x >> 8);
      b[3 * k + 2] = (uint8_t)x;
    }
    const uint64_t at = 3ull * g4;
    const uint32_t nb = (uint32_t)min<uint64_t>(12, 3ull * (groups - g4));
    if (nb == 12 && at + 12 <= limit && (reinterpret_cast<uintptr_t>(o + at) & 3u) == 0) {
      uint32_t* d = reinterpret_cast<uint32_t*>(o + at);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        d[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
               ((uint32_t)b[4 * k + 3] << 24);
    } else {
      for (uint32_t k = 0; k < nb && at + k < limit; ++k) o[at + k] = b[k];
    }
  }
  if (threadIdx.x == 0) {
    if (extra) {
      const uint32_t a = 4 * groups;
      const uint32_t x = ((uint32_t)s[a] << 18) | ((uint32_t)s[a + 1] << 12) |
                         ((uint32_t)(extra == 2 ? s[a + 2] : 0) << 6);
      const uint64_t at = 3ull * groups;
      if (at < limit) o[at] = (uint8_t)(x >> 16);
      if (extra == 2 && at + 1 < limit) o[at + 1] = (uint8_t)(x >> 8);
    }
    sizes[i] = (uint32_t)min<uint64_t>(want, limit);
    over[i] = want > limit ? 1 : 0;
  }
  // the rest of the slot: zeros, never stale device bytes (lbf_b64_verify_batch copies whole slots back)
  for (uint64_t p = want + threadIdx.x; p < limit; p += kB64Threads) o[p] = 0;
}

}  // namespace
}  // namespace lbf

namespace lbf {
namespace {

// ---------------------------------------------------------------------------
// The sender's base64 encode (lbf_verify_encode_b64_batch): the text a
// SendChunk frame carries for chunk i, written as xmlrpc++ 0.7's encoder
// writes it (base64.h:154-210) and as the frame sends it (CR/LF become spaces,
// PeerConnection.cpp:132-156): four characters per three bytes, a space after
// every 18th complete group, the last one or two bytes as "xx==" / "xxx=".
// Group g of chunk i lands at 4g + g/18, so every lane writes its groups
// independently.  blockIdx.x = chunk; data[data_off[i] .. + size[i]) ->
// text[text_off[i] .. + b64_put_length(size[i])).
// ---------------------------------------------------------------------------
__host__ __device__ constexpr uint64_t b64_put_length(uint64_t size) {
  return 4 * (size / 3) + (size % 3 ? 4 : 0) + size / 3 / 18;
}

// One tile of the encode from its bytes in LDS (sb, from byte `delta`): lane
// v writes characters [16v, 16v + 16) of the tile's text.  Characters [p, p +
// 16) of a line lie in at most five consecutive "words" of the line's
// character stream, where word e of line l is group e's four characters for
// e < 18 and, past the line's end, the next line's group e - 18 shifted one
// byte right behind the separator; v_alignbyte cuts the block out of them.
// kWhole: every group of the tile is a whole group of the chunk (all tiles but
// a chunk's last), so no group needs the end-of-text checks; characters a
// block's window computes past the tile come from stale LDS and are cut away.
// That and one v_perm_b32 for the group's byte order took the encode from
// 120.2-121.4 to 101.9-102.4 us per 1,024 x 256 KiB (alternating traces,
// profiles/r05/b64_geometry/ab_traces_enc_whole.json).
template <bool kWhole>
__device__ __forceinline__ void b64_encode_tile(const uint8_t* sb, uint32_t delta, const uint8_t* alpha,
                                                uint32_t tile, uint32_t full, uint32_t rest, uint64_t tl,
                                                uint8_t* t) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(sb);
  const uint32_t tbeg = tile * kB64TileText;
  // group gl of the tile as its four characters, first character in the low byte
  auto chars = [&](uint32_t gl) -> uint32_t {
    const uint32_t gg = tile * kB64TileGroups + gl;
    if (!kWhole && (gg > full || (gg == full && rest == 0))) return 0u;  // past the text
    const uint32_t b = lds_u32_at(w, delta + 3 * gl);
    uint32_t x = __builtin_amdgcn_perm(0u, b, 0x0C000102u);  // the group's three bytes, big-endian
    if (kWhole || gg < full)
      return (uint32_t)alpha[x >> 18] | (uint32_t)alpha[(x >> 12) & 63] << 8 | (uint32_t)alpha[(x >> 6) & 63] << 16 |
             (uint32_t)alpha[x & 63] << 24;
    x &= rest == 2 ? 0xFFFF00u : 0xFF0000u;  // the last one or two bytes: "xxx=" / "xx=="
    return (uint32_t)alpha[x >> 18] | (uint32_t)alpha[(x >> 12) & 63] << 8 |
           (rest == 2 ? (uint32_t)alpha[(x >> 6) & 63] : (uint32_t)'=') << 16 | (uint32_t)'=' << 24;
  };
  for (uint32_t v = threadIdx.x; v < kB64TileText / 16; v += kB64Threads) {
    const uint32_t p0 = 16 * v;
    const uint64_t pos = tbeg + p0;
    if (pos >= tl) break;
    const uint32_t line = p0 / 73, col = p0 - 73 * line, e0 = col >> 2;
    uint32_t g[5], E[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) g[k] = chars(18 * line + e0 + k);
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint32_t e = e0 + k;
      // past the line's 18 groups: the separator, then the next line's characters one byte right
      E[k] = e <= 17 ? g[k] : (g[k] << 8) | (e == 18 ? (uint32_t)' ' : (k > 0 ? g[k - 1] >> 24 : 0u));
    }
    const uint32_t sh = col & 3;
    const uint4 out = make_uint4(__builtin_amdgcn_alignbyte(E[1], E[0], sh), __builtin_amdgcn_alignbyte(E[2], E[1], sh),
                                 __builtin_amdgcn_alignbyte(E[3], E[2], sh), __builtin_amdgcn_alignbyte(E[4], E[3], sh));
    b64_put_block(t, pos, tl, out);
  }
}

// blockIdx.x = group of tiles, blockIdx.y = chunk - chunk0: tile k of chunk i
// encodes bytes [3456k, +3456) into text [4672k, +4672) (clipped to the
// chunk), kEncTilesPerGroup tiles per workgroup, double-buffered as the decode.
__global__ void __launch_bounds__(kB64Threads) b64_encode_kernel(const uint8_t* __restrict__ data,
                                                                 const uint64_t* __restrict__ data_off,
                                                                 const uint32_t* __restrict__ size,
                                                                 uint8_t* __restrict__ text,
                                                                 const uint64_t* __restrict__ text_off, uint32_t tiles,
                                                                 uint32_t chunk0) {
  // a tile's span, its phase, and slack for the group reads of the last window
  // (computed for every word, used only inside the tile)
  constexpr uint32_t kStage = (kB64TileBytes + 15) / 16 + 4;
  constexpr uint32_t kPer = (kStage + kB64Threads - 1) / kB64Threads;  // staged blocks per lane
  __shared__ uint4 stage[2][kStage];
  __shared__ uint8_t alpha[64];
  const uint32_t i = chunk0 + blockIdx.y, t0 = blockIdx.x * kEncTilesPerGroup;
  const uint32_t n = size[i], full = n / 3, rest = n % 3;
  const uint64_t tl = b64_put_length(n);
  const uint32_t own = (uint32_t)((tl + kB64TileText - 1) / kB64TileText);
  if (t0 >= own) return;  // the whole workgroup: no barrier below is reached
  const uint32_t t1 = min(own, t0 + kEncTilesPerGroup);
  const uint8_t* d = data + data_off[i];
  uint8_t* t = text + text_off[i];
  B64Stage<kPer> st;
  auto load = [&](uint32_t tile) {
    const uint32_t dbeg = tile * kB64TileBytes;
    st.blocks = 0;
    st.delta = 0;
    if (dbeg < n) st.load(d + dbeg, min(kB64TileBytes, n - dbeg));
  };
  load(t0);
  if (threadIdx.x < 64) {
    const uint32_t c = threadIdx.x;
    alpha[c] = (uint8_t)(c < 26 ? 'A' + c : c < 52 ? 'a' + (c - 26) : c < 62 ? '0' + (c - 52) : c == 62 ? '+' : '/');
  }
  st.store(stage[0]);
  uint32_t delta = st.delta;
  __syncthreads();
  for (uint32_t tile = t0; tile < t1; ++tile) {
    const uint32_t buf = (tile - t0) & 1u;
    if (tile + 1 < t1) load(tile + 1);  // in flight while this tile encodes
    if ((tile + 1) * kB64TileGroups <= full)  // uniform over the workgroup
      b64_encode_tile<true>(reinterpret_cast<const uint8_t*>(stage[buf]), delta, alpha, tile, full, rest, tl, t);
    else
      b64_encode_tile<false>(reinterpret_cast<const uint8_t*>(stage[buf]), delta, alpha, tile, full, rest, tl, t);
    if (tile + 1 < t1) {
      st.store(stage[buf ^ 1u]);
      delta = st.delta;
      __syncthreads();
    }
  }
}

}  // namespace
}  // namespace lbf
