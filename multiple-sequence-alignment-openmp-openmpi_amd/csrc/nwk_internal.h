// nwk_internal.h -- shared between the HIP kernels and the host runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nwk {

constexpr int kWave = 64;
constexpr int kRows = 8;                  // DP rows per lane (R)
constexpr int kBandRows = kWave * kRows;  // rows per band = one wave's task
constexpr int kEPad = 128;                // E / SEL entries before column 0
constexpr int kETail = 384;               // E / SEL entries past the last column
// Sequence-code buffer padding.  The traceback stages 256-byte windows by
// LDS-DMA: y windows start up to 96 bytes before a sequence, x windows end up
// to ~660 bytes past the last 512-row band's first row.
constexpr int kCodesFrontPad = 256;
constexpr int kCodesTailPad = 1024;

// Recurrence variants (see DESIGN.md "Kernels").
enum Mode : int {
  kProfile = 0,  // |alphabet| <= 4, penalties >= 0: signed-byte substitution profile
  kCompare = 1,  // any bytes, penalties >= 0: byte compare + select
  kLiteral = 2,  // any penalties: skel:215-224 literally (match ? diag : min3)
  kAffine = 3,   // affine gaps: 4-bit traceback codes, compare mode
  kPacked = 4,   // kProfile at W = 4 with two cells per register (int16 pairs), packed layout
  kPacked2 = 5,  // kPacked with two bands per wave (band pairs), layout LY 2
  kProfileDP = 6,  // profile-profile sum-of-pairs DP of the progressive MSA, 4-bit codes
  kAffinePk = 7,   // kAffine on band pairs as int16 pairs (nw_align_pka), layout LY 2, profile codes
  kBits = 8,       // bit-sliced difference planes (nw_align_bits, nwk_bits.hip): 2048-row bands, 2-bit traceback
  kBitsStrip = 9,  // kBits as rolling strips (nw_align_strip): one wave per pair, every band in turn
  kCol = 10,       // bit-parallel columns (nw_align_col, nwk_col.hip): kBits' domain and storage, a pair's span n + ~96 x bands
  kGotoh = 11,     // affine gaps as bit-sliced thermometer planes (nw_align_gotoh, nwk_gotoh.hip): 2048-row bands,
                   // four traceback words per step (D, F-source, E-extend, F-extend), fused device walk
};
constexpr int kBitsRows = 2048;  // kBits: rows per band (64 lanes x 32 bits)

// kGotoh geometry (nw_align_gotoh): lane t bit b holds row 32 t + b of a
// 2048-row band, at (1-based) column s - 32 t - b at step s.  Storage: 4-step
// blocks of 1024 dwords, word w (0 D, 1 F-source, 2 E-extend, 3 F-extend) of
// step s, lane t at w * 256 + (s & 2) * 64 + 2 t + (s & 1).  Windowed
// (bits_w > 0): band b keeps blocks gotoh_blk_lo(b) .. + bits_nblk, the steps
// of its cells within bits_w columns of the diagonal j = i n / m.
__host__ __device__ inline int gotoh_blk_lo(int b, int m, int n, int w) {
  if (w <= 0) return 0;
  const int64_t lo = (int64_t)b * kBitsRows * n / m - w;
  return lo <= 0 ? 0 : (int)(lo >> 2);
}

// One pair of the batch.  All offsets are element offsets into the
// batch-level arrays passed to the kernels.
struct PairDesc {
  int64_t x_off;    // codes of x (DP rows) in `codes`
  int64_t y_off;    // codes of y (DP columns) in `codes`
  int64_t e_off;    // E index of y's column-0 entry (E[e_off + a] packs y[a..a+3])
  int64_t mat_off;  // first dword of this pair's stored matrix
  int64_t bnd_off;  // first granule of this pair's band-boundary rows
  int64_t ops_off;  // first byte of this pair's traceback op buffer (capacity m+n)
  int32_t m, n;
  int32_t nbands;   // ceil(m / kBandRows)
  int32_t nchunks;  // ceil(n / 64): 64-column boundary chunks
  int32_t sblocks;  // 64-step super-blocks per band = nchunks + 1 (kPacked: + 2)
  int32_t slot;     // index of this pair in the batch's result arrays
  // kPacked / kPacked2 segmented traceback (see run_segments / nw_gather)
  int32_t spec_every;   // a speculative segment after every spec_every-th task (0: whole-pair trace)
  int32_t nguess;       // start columns per speculative boundary (segment id = task * nguess + guess)
  int64_t task_off;     // first entry of this pair in tdone (one per task)
  int64_t seg_off;      // first entry of this pair in seginfo (tasks * nguess)
  int64_t rec_off;      // first record of this pair in recs ([m / 128 + 1][2])
  int64_t segops_off;   // first byte of this pair's segment move buffers in segops
  // linear-space traceback group (FillArgs.lin_mode 2): bands in the group,
  // trace start cell, row where the trace stops (the group's top)
  int32_t lin_nb, lin_i, lin_j, lin_stop;
  // Windowed storage (kBits, kAffinePk): only the steps within bits_w columns
  // of the pair's diagonal j = i n / m are stored (bits_w = 0: all of them).
  // kBits: bits_nblk 8-step blocks per band (band b keeps blocks
  // bits_blk_lo(b) ..); kAffinePk: bits_nblk 64-step super-blocks per band
  // pair (band pair p keeps super-blocks pka_sb_lo(p) ..).
  int32_t bits_w, bits_nblk;
  // kBitsStrip: columns per row pass n' (a multiple of 64, >= n + 32): one
  // wave sweeps all bands of the pair as a rolling 2048-row strip -- lane bit p
  // runs rows p, p + 2048, ... with virtual column v = s - p, pass v / n',
  // column v % n' (0 = banded tasks)
  int32_t bits_np;
  int32_t prio;     // kCol: issue priority (s_setprio) of the pair's fill tasks -- the longest spans of a span-bound batch
  int64_t xw_off;   // kBitsStrip: y-window index of the row sequence's position 0 (its row codes)
};

// kBits: first stored 8-step block of band b (see PairDesc::bits_w)
__host__ __device__ inline int bits_blk_lo(int b, int m, int n, int w) {
  if (w <= 0) return 0;
  const int64_t lo = (int64_t)b * kBitsRows * n / m - w;
  return lo <= 0 ? 0 : (int)(lo >> 3);
}

// kBits / kBitsStrip windowed storage below one band's height: only the lane
// words holding a cell within w columns of the diagonal are written (and the
// traceback checks every cell against that); at w >= 2048 nearly every lane
// word of a stored block holds such a cell, so all are written
__host__ __device__ inline bool bits_lane_window(int w) { return w > 0 && w < kBitsRows; }

// kCol segmented traceback (PairDesc::spec_every > 0; nwk_col.hip trace_col):
// for each band b < nbands - 1 of a pair, its speculative segment's
//   records  u64 [2048] at recs + rec_off + 2048 b: row rr's entry cell
//            {epoch & 0xfffff : 20 | column : 22 | move index : 22}
//   info     int4 at seginfo + 4 (seg_off + b): {flag = epoch once done,
//            length (-1: failed), exit row (absolute), exit column}
//   moves    u8 [colseg_cap(n)] at segops + segops_off + b cap
__host__ __device__ inline int64_t colseg_cap(int n) { return ((int64_t)kBitsRows + n + 64 + 16 + 127) / 128 * 128; }
// record fields: 22-bit column and move index (a band's segment has < 2048 + n + 64 moves)
__host__ __device__ inline bool colseg_ok(int n) { return (int64_t)kBitsRows + n + 64 < (1 << 22); }

// kBitsStrip: first stored 8-step block (strip step numbering) of band b's
// window: its cells (i, j), |j - i n / m| <= w, sit at steps j + b np + (i - 2048 b)
__host__ __device__ inline int strip_blk_lo(int b, int m, int n, int np, int w) {
  if (w <= 0) return 0;
  const int64_t lo = (int64_t)b * np + (int64_t)b * kBitsRows * n / m - w;
  return lo <= 0 ? 0 : (int)(lo >> 3);
}

// kAffinePk: first stored super-block of band pair p.  Its rows R+1 .. R+1024
// (R = 1024 p) put cell (i, j) of half h, lane t at step j - 1 + t + 64 h, so
// the window's cells j >= i n / m - w sit at steps >= R n / m - w - 1.
__host__ __device__ inline int pka_sb_lo(int p, int m, int n, int w) {
  if (w <= 0) return 0;
  const int64_t lo = (int64_t)p * 2 * kBandRows * n / m - w - 64;
  return lo <= 0 ? 0 : (int)(lo >> 6);
}

struct FillArgs {
  const PairDesc* pairs;
  const int2* tasks;       // {pair index, band}, dependency-ordered
  int ntasks;
  const uint8_t* codes;    // sequence codes (x rows, y columns)
  const uint32_t* E;       // expanded column codes, 4 per dword
  const uint32_t* sel;     // kPacked: per column v_perm selector {y[a], hi, 4+y[a-1], hi}; kPacked2: {y[a], hi, 4+y[a-64], hi}
  uint32_t* mat;           // packed G = H - (i+j)*pgap, W bits per cell
  unsigned long long* bnd; // {epoch:32 | G:32} granules, one per boundary cell
  unsigned* counter;       // task dequeue head
  unsigned* err;           // nonzero = a hand-off timed out
  unsigned* done;          // per slot: bands finished (released at agent scope)
  uint8_t* ops;            // per pair, reversed traceback moves: 'D','U','L'
  int* oplen;              // per slot
  int2* endij;             // per slot: (i, j) where the traced walk stopped
  unsigned long long* stamps;  // optional (verbose >= 2): per-slot diagnostics (see nwk_runtime.cpp)
  int ntasks_pairs;            // pairs in the batch (diagnostic layout)
  unsigned epoch;
  int K0, K1;              // diag increments in G-space: match, mismatch (kAffine: K1 = pxy)
  int go, ge;              // kAffine: gap open / extend
  int dbg_notrace;         // debug: skip the affine traceback
  int dbg_badwalk;         // debug (tests): slot + 1 whose nw_align_col walk reports itself failed (err 16)
  int band_prio;           // kCol: issue priority by band (upstream bands first): 0 off, 1 on
  int lin_mode;            // nw_align: 0 normal, 1 linear-space fill pass, 2 linear-space group recompute + trace
  unsigned* prog;          // debug: per-wave progress markers (NWK_WATCHDOG)
  unsigned* tdone;         // kPacked2: per task, 1 = filled and released
  int* seginfo;            // kPacked2: per task, 8 ints {len, ei, ej, mseg, midx, off lo, off hi, -}
  unsigned long long* recs;  // kPacked2: traceback record rows
  uint8_t* segops;         // kPacked2: segment move buffers
  int2* tjobs;             // queued extra guesses {pair, segment id}
  unsigned* tj_ready;      // per job: 1 = written
  unsigned* tj_head;       // consumer counter
  unsigned* tj_tail;       // producer counter
  int ntjobs;              // jobs the batch will produce
  const int* prow;         // kProfileDP: per X column (DP row) 8 ints {rc[0..5], gx, H[i][0]} at pairs[].x_off
  const int* pcol;         // kProfileDP: per Y column (DP column) 8 ints {cnt[0..5], gy, H[0][j]} at pairs[].y_off
  const unsigned* yw;      // kBits: per y position p two dwords (code bit planes of y[p .. p+31], y[p] at bit 31), at pairs[].e_off
  int* retry;              // windowed storage: per slot, 1 = the path left the stored window (re-run in full)
  int strip_ring;          // kBitsStrip: LDS dwords per wave of the hand-off ring (max n' / 64 x 2 NP)
  // Fused pair finalize (kBits / kBitsStrip with device finalize, nwk_bits.hip):
  // the wave that traced a pair writes its rows and penalty (whole wave) and
  // queues the pair; a wave that finds >= 32 queued pairs (or, once the fill
  // tasks are gone, any) hashes them one row per lane, as nw_hash does, and
  // writes the records {penalty, problemhash} and then fin_flag[slot] = epoch
  // into host-mapped memory, so the host takes results during the launch.
  int fuse_fin;
  int pxy, pgap;           // linear move costs (penalty sum)
  const uint8_t* raw;      // raw sequence bytes (codes layout)
  int64_t ops_base;        // rows sit at rows1/2 + (ops_off - ops_base)
  uint8_t* rows1;
  uint8_t* rows2;
  int* fin_len;            // per slot (device): row length, then the penalty at [np + slot]
  unsigned long long* hq;  // queue of traced pairs: {epoch:32 | slot:32}, np entries
  unsigned* hq_ctl;        // [0] entries reserved, [1] entries claimed, [2] pairs traced, [3] drain waves
  int* fin_pen;            // per slot (host-mapped)
  uint8_t* fin_hash;       // per slot, 64 raw bytes (host-mapped)
  unsigned* fin_flag;      // per slot (host-mapped): = epoch once the record is written
  // Streamed host finalize (kCol, host-side finalize): the pair walk writes
  // its moves to host-mapped ops_host + (ops_off - ops_base) and then, per
  // slot, host_rec {flag = epoch, length (-1: left the window, -2: the walk failed), end i, end j}
  // (flag last, system scope), so host threads finalize pairs during the launch.
  uint8_t* ops_host;
  int* host_rec;
  // Fill-vs-walk guard (skel:274 `ret = dp[m][n]`): per slot, the fill's own
  // H(m, n), accumulated by the band tasks with agent-scope atomic adds onto a
  // zeroed word before they release (bit-plane kernels: -sum of the vertical
  // differences down column n per band, plus the border term; value kernels:
  // the cell itself).  Every finalize compares it with the cost of the walked
  // path and re-runs a pair that disagrees (retry[slot] = 2) instead of
  // publishing it.  nullptr: the kernel does not provide it.
  int* endv;
  int dbg_corrupt;         // debug (tests): slot + 1 whose stored code of cell (m, n) is flipped before its walk
  // fused finalize of a streamed shard: a pair of PairDesc::prio >= early_hash
  // (the first pieces of the canonical order) is hashed by its tracing wave at
  // once instead of waiting for a group of 32 (0: off)
  int early_hash;
};
// host_rec ints per slot: {flag, length, end i, end j, fill end value H(m, n), -, -, -}
constexpr int kHostRecInts = 8;
constexpr int kProfSyms = 6;  // kProfileDP: symbols + gap per column profile

constexpr int kMaxSegsPerPair = 16384;  // segment ids are 14 bits in the traceback records

// Device pair finalize (nwk_hash.hip): rows, penalty, problemhash per pair.
struct HashArgs {
  const PairDesc* pairs;
  int npairs;
  const uint8_t* raw;      // raw sequence bytes (codes layout)
  const uint8_t* ops;      // traced moves per pair (reversed), at pairs[].ops_off
  int64_t ops_base;        // byte offset of the op region: pair rows sit at rows1/2 + (ops_off - ops_base)
  uint8_t* rows1;          // align1 rows (16-aligned per pair, op-region layout, + 256 B slack)
  uint8_t* rows2;          // align2 rows
  const int* oplen;        // per slot
  const int2* endij;       // per slot
  int pxy, gopen, gext;    // move costs (linear: gopen = gext = pgap)
  int* penalties;          // per slot
  uint8_t* hashes;         // per slot, 64 raw bytes
  const int* endv;         // per slot: the fill's H(m, n) (FillArgs::endv), nullptr = unchecked
  int* retry;              // per slot: set to 2 when the walked path's cost differs from endv
};
hipError_t launch_hash(const HashArgs& h, hipStream_t s);

// Launchers (nwk_kernels.hip).  bits in {4, 8, 16, 32}.
hipError_t launch_fill(int mode, int bits, const FillArgs& a, int grid, hipStream_t s);
hipError_t launch_gather(const FillArgs& a, int npairs, int task_shift, hipStream_t s);
int fill_blocks_per_cu(int mode, int bits);
// kBits (nwk_bits.hip)
bool bits_admissible(int pxy, int pgap, int alpha);
hipError_t launch_bits(const FillArgs& a, int pxy, int pgap, int grid, hipStream_t s);
int bits_blocks_per_cu(int pgap);
hipError_t launch_strip(const FillArgs& a, int pxy, int pgap, int grid, hipStream_t s);
int strip_blocks_per_cu(int pgap, int ring_dwords);
// kCol (nwk_col.hip)
// hi: the plain instantiation at NWK_COL_WPE_HI waves per SIMD (not with fuse_fin)
hipError_t launch_col(const FillArgs& a, int pxy, int pgap, int grid, bool hi, hipStream_t s);
int col_blocks_per_cu(int pgap, bool hi = false);
// kGotoh (nwk_gotoh.hip): instantiated for a fixed set of (pxy, go, ge)
bool gotoh_admissible(int pxy, int go, int ge, int alpha);
int gotoh_granules(int go, int ge);  // granules per 32-column chunk of a band's last row
hipError_t launch_gotoh(const FillArgs& a, int pxy, int go, int ge, int grid, hipStream_t s);
int gotoh_blocks_per_cu(int pxy, int go, int ge);

// Dwords of one band of the stored matrix.
__host__ __device__ inline int64_t band_dwords(int bits, int sblocks) {
  const int spd = 32 / bits;  // steps per dword
  return (int64_t)sblocks * (64 / spd) * kRows * kWave;
}

}  // namespace nwk
