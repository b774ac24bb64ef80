// nwk_hash.hip -- device-side pair finalize: alignment rows, penalty and
// problemhash.
//
// Reference (skel = testing3/seqalign-mpi-skeleton.cpp):
//   prefix fill skel:263-272, trim skel:135-154, strings skel:146-154,
//   problemhash = sha512hex(sha512hex(align1) ++ sha512hex(align2)) skel:155-157,
//   sha512 = sw::sha512::calculate (sha512.hh:159-164, FIPS 180-4).
//
// nw_rows materialises align1 / align2 of every pair in HBM (coalesced,
// wave-scan based, one workgroup per pair) and sums the path cost (= dp[m][n], the
// reference's penalty); nw_hash then runs one lane per row over 16-byte loads
// (SHA-512 is sequential within a message), and the two digests meet through
// a lane shuffle so the even lane can hash their 256 hex characters.  Valid when no input byte is
// '_' (then no column is '_' in both rows and the trim keeps everything; the
// host checks and otherwise finalizes on the CPU).
#include "nwk_internal.h"
#include "nwk_sha_dev.h"

namespace nwk {

using namespace shadev;

// Rows + penalty, one workgroup per pair (skel:263-272 prefix, then the traced
// moves in forward order).  Wave w of the four owns a contiguous quarter of the
// forward moves.  Pass 1 counts the quarter's x / y advances; pass 2 walks it
// 64 moves per iteration, lane l taking move base + l: one coalesced 64-byte
// read of the (reversed) move string, a wave scan of the packed advances
// {x | y << 16} for each lane's x / y index, coalesced 64-byte row writes.
// (The first version gave each of 256 threads a private ~400-move chunk read
// byte by byte: every load touched 256 lines, 7 ms on C3.)
__global__ __launch_bounds__(256) void nw_rows(HashArgs h) {
  __shared__ int tx[4], ty[4];
  __shared__ long long sp[4];
  const int q = blockIdx.x;
  const PairDesc pd = h.pairs[q];
  const int nops = h.oplen[pd.slot];
  const int2 e = h.endij[pd.slot];
  const int pre = e.x > 0 ? e.x : e.y;
  const uint8_t* ops = h.ops + pd.ops_off;
  const uint8_t* x = h.raw + pd.x_off;
  const uint8_t* y = h.raw + pd.y_off;
  uint8_t* r1 = h.rows1 + (pd.ops_off - h.ops_base);
  uint8_t* r2 = h.rows2 + (pd.ops_off - h.ops_base);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int t = tid; t < pre; t += 256) {  // prefix run
    r1[t] = e.x > 0 ? x[t] : (uint8_t)'_';
    r2[t] = e.x > 0 ? (uint8_t)'_' : y[t];
  }
  const int Q = ((nops + 3) / 4 + 63) & ~63;  // moves per wave, whole iterations
  const int F0 = min(nops, w * Q), F1 = min(nops, F0 + Q);
  // pass 1: this quarter's advances
  int cx = 0, cy = 0;
  for (int f = F0 + lane; f < F1; f += 64) {
    const unsigned op = ops[nops - 1 - f];
    const bool d = op == 'D', up = op == 'U' || op == 'u';
    cx += (d || up) ? 1 : 0;
    cy += (d || !up) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    cx += __shfl_xor(cx, o);
    cy += __shfl_xor(cy, o);
  }
  if (lane == 0) { tx[w] = cx; ty[w] = cy; }
  __syncthreads();
  int ix = e.x, iy = e.y;
  for (int v = 0; v < w; ++v) { ix += tx[v]; iy += ty[v]; }
  // pass 2
  long long pen = 0;
  for (int base = F0; base < F1; base += 64) {
    const int f = base + lane;
    const bool live = f < F1;
    const unsigned op = live ? ops[nops - 1 - f] : 0u;
    const bool d = op == 'D', up = op == 'U' || op == 'u';
    const bool ax = live && (d || up), ay = live && (d || !up);
    const unsigned adv = (ax ? 1u : 0u) | (ay ? 0x10000u : 0u);
    const unsigned inc = wave_incl_scan(adv, lane);
    const unsigned exc = inc - adv;
    if (live) {
      const unsigned chx = ax ? x[ix + (int)(exc & 0xffffu)] : (unsigned)'_';
      const unsigned chy = ay ? y[iy + (int)(exc >> 16)] : (unsigned)'_';
      r1[pre + f] = (uint8_t)chx;
      r2[pre + f] = (uint8_t)chy;
      pen += d ? (chx == chy ? 0 : h.pxy) : (op == 'u' || op == 'l' ? h.gopen : h.gext);
    }
    const unsigned tot = (unsigned)__shfl((int)inc, 63);
    ix += (int)(tot & 0xffffu);
    iy += (int)(tot >> 16);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pen += __shfl_xor(pen, o);
  if (lane == 0) sp[w] = pen;
  __syncthreads();
  if (tid == 0) {
    const int p = (int)(sp[0] + sp[1] + sp[2] + sp[3] + (pre > 0 ? h.gopen + (long long)(pre - 1) * h.gext : 0));
    h.penalties[pd.slot] = p;
    // the fill-vs-walk guard (skel:274): a walk that read a wrong code gives a
    // path whose cost is not the fill's H(m, n) -- never published, re-run
    // (a pair whose walk left its storage window, retry 1, has no path here)
    if (h.endv && h.retry[pd.slot] == 0 && p != h.endv[pd.slot]) h.retry[pd.slot] = 2;
  }
}

// SHA-512 of one materialised row per lane (lane 2q: align1 of pair q, lane
// 2q+1: align2), 128-byte blocks by 16-byte loads with the next block in
// flight behind this block's rounds; then the even lane hashes the two
// digests' hex (skel:155-157).
__global__ __launch_bounds__(256) void nw_hash(HashArgs h) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  const int q = tid >> 1, side = tid & 1;
  const bool live = q < h.npairs;
  const PairDesc pd = h.pairs[live ? q : 0];
  const int nops = live ? h.oplen[pd.slot] : 0;
  const int2 e = live ? h.endij[pd.slot] : make_int2(0, 0);
  const int64_t L = live ? (int64_t)(e.x > 0 ? e.x : e.y) + nops : 0;
  const uint4* row = reinterpret_cast<const uint4*>((side ? h.rows2 : h.rows1) + (pd.ops_off - h.ops_base));
  Sha sh;
  sh.init();
  const int64_t nblk = (L + 17 + 127) / 128;
  int64_t wblk = nblk;  // per wave: as many blocks as its longest row
  for (int o = 32; o > 0; o >>= 1) wblk = max(wblk, (int64_t)__shfl_xor(wblk, o));
  const int64_t ndata = (L + 127) / 128;  // blocks holding message bytes (readable: row buffers are padded)
  uint4 cur[8], nxt[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) cur[k] = ndata > 0 ? row[k] : make_uint4(0, 0, 0, 0);
  for (int64_t bk = 0; bk < wblk; ++bk) {
#pragma unroll
    for (int k = 0; k < 8; ++k) nxt[k] = bk + 1 < ndata ? row[8 * (bk + 1) + k] : make_uint4(0, 0, 0, 0);
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // little-endian dwords -> big-endian 64-bit words
      w[2 * k] = ((uint64_t)__builtin_bswap32(cur[k].x) << 32) | __builtin_bswap32(cur[k].y);
      w[2 * k + 1] = ((uint64_t)__builtin_bswap32(cur[k].z) << 32) | __builtin_bswap32(cur[k].w);
    }
    const int64_t b0 = 128 * bk;  // message bytes [b0, b0+128)
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // clear bytes past L, place the 0x80 terminator
      const int64_t s0 = b0 + 8 * k;
      if (s0 + 8 > L) {
        const int keep = (int)max((int64_t)0, min((int64_t)8, L - s0));
        uint64_t v = keep > 0 ? w[k] & (~0ull << (64 - 8 * keep)) : 0ull;
        if (L >= s0 && L < s0 + 8) v |= 0x80ull << (56 - 8 * (L - s0));
        w[k] = v;
      }
    }
    if (bk == nblk - 1) w[15] = (uint64_t)L * 8u;
    if (bk < nblk) sh.block(w);
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = nxt[k];
  }
  uint64_t other[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) other[k] = __shfl_xor(sh.s[k], 1);
  if (!live || side != 0) return;
  Sha p;
  p.init();
  uint64_t w[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[2 * k] = hex16((uint32_t)(sh.s[k] >> 32));
    w[2 * k + 1] = hex16((uint32_t)sh.s[k]);
  }
  p.block(w);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w[2 * k] = hex16((uint32_t)(other[k] >> 32));
    w[2 * k + 1] = hex16((uint32_t)other[k]);
  }
  p.block(w);
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = 0;
  w[0] = 0x8000000000000000ULL;
  w[15] = 256 * 8;
  p.block(w);
  uint8_t* out = h.hashes + 64 * (int64_t)pd.slot;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t v = p.s[k];
#pragma unroll
    for (int b = 0; b < 8; ++b) out[8 * k + b] = (uint8_t)(v >> (56 - 8 * b));
  }
}

hipError_t launch_hash(const HashArgs& h, hipStream_t s) {
  if (h.npairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(nw_rows, dim3(h.npairs), dim3(256), 0, s, h);
  const int threads = 2 * h.npairs;
  hipLaunchKernelGGL(nw_hash, dim3((threads + 255) / 256), dim3(256), 0, s, h);
  return hipGetLastError();
}

}  // namespace nwk
