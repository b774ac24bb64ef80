// nwk_runtime.cpp -- host side of the C-ABI in include/nwk.h.
//
// Replaces, for the hot path of the reference (paths relative to the
// reference repository):
//   getMinimumPenalties / do_MPI_task / do_task   submit/xuliny-seqalkway.cpp:183-417
//   trim + string build + hashes                  seqalign-mpi-skeleton.cpp:135-159
// The MPI master/worker queue becomes: canonical pair ids -> HBM-budgeted
// batches -> one persistent fill launch + one traceback launch per batch per
// device -> host trim/SHA-512 on a thread pool -> (multi-GPU) one
// ncclAllGather of 72-byte result records -> rank-0 hash chain.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>
#include <unistd.h>

#include "../../include/nwk.h"
#include "nwk_internal.h"
#include "nwk_prof.h"
#include "sha512.h"

using namespace nwk;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t e_ = (expr);                                                                \
    if (e_ != hipSuccess)                                                                  \
      return fail(e_ == hipErrorOutOfMemory ? NWK_ENOMEM : NWK_EDEVICE, "%s: %s (%s:%d)", \
                  #expr, hipGetErrorString(e_), __FILE__, __LINE__);                       \
  } while (0)

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t round_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

// Canonical pair id -> (i, j), skel:122-123.
inline void pair_ij(int64_t p, int* i, int* j) {
  int64_t ii = (int64_t)((1.0 + std::sqrt(1.0 + 8.0 * (double)p)) / 2.0);
  while (ii * (ii - 1) / 2 > p) --ii;
  while ((ii + 1) * ii / 2 <= p) ++ii;
  *i = (int)ii;
  *j = (int)(p - ii * (ii - 1) / 2);
}

// Device buffer that only grows.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return NWK_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(hipMalloc(&p, bytes));
    cap = bytes;
    // debug: NWK_POISON=<byte> fills fresh device buffers, so a read of memory no
    // kernel or copy has written shows up as a wrong answer on every run
    // (buffers of at least NWK_POISON_MIN bytes; the fill completes before the
    // engine's own stream uses the buffer)
    static const int poison = getenv("NWK_POISON") ? atoi(getenv("NWK_POISON")) : -1;
    static const long long poison_min = getenv("NWK_POISON_MIN") ? atoll(getenv("NWK_POISON_MIN")) : 0;
    if (poison >= 0 && (long long)bytes >= poison_min) {
      HIP_TRY(hipMemset(p, poison & 0xff, bytes));
      HIP_TRY(hipDeviceSynchronize());
    }
    return NWK_OK;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes, unsigned flags = hipHostMallocDefault) {
    if (bytes <= cap) return NWK_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(hipHostMalloc(&p, bytes, flags));
    cap = bytes;
    return NWK_OK;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return static_cast<T*>(p); }
};

struct PairWork {
  int64_t id;       // canonical pair id
  int64_t out;      // index in the caller's output arrays
  int i, j;         // x = seq i (rows), y = seq j (columns)
  int m, n;
  int64_t mat_dw, bnd_gr, ops_b;  // footprint
  int64_t segops_b, segctl_b;     // kPacked2 segmented traceback: move buffers, control (flags, info, records)
  int spec;                       // segmented traceback: spec_every
  int nguess;                     // segmented traceback: start columns per speculative boundary
  int64_t njobs;                  // queued extra guesses (spec boundaries x (nguess - 1))
  int bits_w = 0;                 // kBits windowed storage: half-width in columns (0 = full), see PairDesc
  int bits_nblk = 0;              // kBits: stored 8-step blocks per band
  int guard = 0;                  // fill-vs-walk guard: times this pair was re-run because its walk disagreed
};

}  // namespace

struct nwk_ctx {
  nwk_opts opts{};
  int device = 0;
  int cus = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {};
  int64_t budget = 0;
  unsigned epoch = 0;
  int host_threads = 1;

  // sequence set
  int k = 0;
  std::vector<int64_t> off;     // k+1
  std::vector<uint8_t> seqs;    // raw bytes
  int alpha = 0;                // distinct bytes
  uint8_t code_of[256] = {};
  std::vector<int64_t> c_off;   // code offset per sequence (8-aligned)
  std::vector<int64_t> e_off;   // E index of column 0 per sequence
  DevBuf d_codes[2];            // [0] profile codes, [1] raw bytes
  DevBuf d_E[2];
  bool built[2] = {false, false};
  DevBuf d_sel[4];              // selector streams: [hi 0x00, hi 0xff] x [kPacked (lag 1), kPacked2 (lag 64)]
  bool built_sel[4] = {false, false, false, false};
  std::vector<int64_t> yw_off;  // kBits: y-window index of position 0 per sequence
  DevBuf d_yw;                  // kBits: 32-column code-plane windows, two dwords per position
  bool built_yw = false;

  // batch buffers
  DevBuf d_work;                // matrices | boundary granules | op strings
  int64_t clean_b = 0;          // leading bytes of d_work holding only zeros / old-epoch granules
  DevBuf d_pairs, d_tasks, d_ctl, d_oplen, d_endij, d_done, d_stamps, d_prog, d_retry;
  DevBuf d_endv;                // fill-vs-walk guard: per slot, the fill's H(m, n) (FillArgs::endv)
  HostBuf h_endv[2];
  DevBuf d_segctl;              // kPacked2: task-done flags | segment info | traceback records; kCol: segment records
  DevBuf d_colinfo;             // kCol: segment info (int4 per segment), cleared per batch
  int64_t colseg_clean_b = 0;   // kCol: leading bytes of d_segctl holding only zeros / kCol records of older epochs
  unsigned colseg_epoch0 = 0;   // kCol: the epoch of the last clear (records' tags wrap after 2^20 launches)
  DevBuf d_pen, d_hash;         // device finalize (nw_hash): per pair penalty, problemhash
  DevBuf d_hq;                  // fused finalize: queue of traced pairs | row lengths and penalties
  DevBuf d_msa[3];              // nwk_msa: row profiles | column profiles | granules, matrices, moves
  HostBuf h_pen[2], h_hash[2];
  bool has_us = false;          // some input byte is '_': trims need the host finalize
  HostBuf h_tasks;
  HostBuf h_pairs[2], h_oplen[2], h_endij[2], h_ops[2];  // double-buffered: batch b+1 runs while b finalizes
  HostBuf h_retry;  // kBits windowed storage: per slot of the last batch, 1 = re-run with full storage
  // fused finalize (bits kernels): host-mapped coherent records the kernel
  // writes per pair as it is traced, {flag u32 [np] | penalty i32 [np] | hash [np][64]}
  HostBuf h_rec[2];
  // streamed host finalize (kCol): host-mapped move strings and per-slot records {flag, length, end i, end j}
  HostBuf h_opsm[2], h_hrec[2];
  // set while an nwk_align_pairs_begin call runs: align_work marks each
  // caller index whose final result is in place (nwk_align_pairs_poll)
  std::atomic<uint8_t>* ready_out = nullptr;

  nwk_stats stats{};

  // nwk_align_pairs_begin / _end: one call in flight on a host thread
  std::thread async;
  bool pending = false;
  std::vector<int64_t> a_ids;
  std::vector<int32_t> a_pen;
  std::vector<uint8_t> a_hash;
  std::unique_ptr<std::atomic<uint8_t>[]> a_ready;
  std::atomic<int> a_finished{0};  // the in-flight call has returned (a_rc is final)
  int a_rc = NWK_OK;
  std::string a_err;
};

extern "C" {

void nwk_opts_default(nwk_opts* o) {
  memset(o, 0, sizeof *o);
  o->device = 0;
  o->ngpus = 1;
}

const char* nwk_last_error(void) { return g_err.c_str(); }

int nwk_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void nwk_ctx_destroy(nwk_ctx* c) {
  if (!c) return;
  if (c->async.joinable()) c->async.join();
  (void)hipSetDevice(c->device);
  for (auto& b : c->d_codes) b.release();
  for (auto& b : c->d_E) b.release();
  for (auto& b : c->d_sel) b.release();
  c->d_yw.release();
  c->d_work.release();
  c->d_pairs.release(); c->d_tasks.release(); c->d_ctl.release();
  c->d_oplen.release(); c->d_endij.release(); c->d_done.release(); c->d_stamps.release(); c->d_retry.release();
  c->h_retry.release();
  c->d_endv.release(); c->h_endv[0].release(); c->h_endv[1].release();
  c->d_segctl.release(); c->d_colinfo.release(); c->d_prog.release(); c->d_pen.release(); c->d_hash.release(); c->d_hq.release();
  for (auto& b : c->d_msa) b.release();
  for (int b = 0; b < 2; ++b) { c->h_pen[b].release(); c->h_hash[b].release(); c->h_rec[b].release(); }
  for (int b = 0; b < 2; ++b) { c->h_opsm[b].release(); c->h_hrec[b].release(); }
  c->h_tasks.release();
  for (int b = 0; b < 2; ++b) {
    c->h_pairs[b].release(); c->h_oplen[b].release(); c->h_endij[b].release(); c->h_ops[b].release();
  }
  for (auto& e : c->ev) if (e) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int nwk_ctx_create(const nwk_opts* opts, nwk_ctx** out) {
  if (!out) return fail(NWK_EINVAL, "nwk_ctx_create: out is NULL");
  *out = nullptr;
  int ndev = nwk_device_count();
  nwk_opts o;
  nwk_opts_default(&o);
  if (opts) o = *opts;
  if (const char* v = getenv("NWK_VERBOSE")) o.verbose = atoi(v);  // debug: diagnostics on stderr
  // option checks first: they need no device
  if (o.finalize < 0 || o.finalize > 3) return fail(NWK_EINVAL, "nwk_ctx_create: finalize must be 0..3");
  if (o.kernel < 0 || o.kernel > 7) return fail(NWK_EINVAL, "nwk_ctx_create: kernel must be 0..7");
  if (o.task_order < 0 || o.task_order > 2) return fail(NWK_EINVAL, "nwk_ctx_create: task_order must be 0..2");
  if (o.bits != 0 && o.bits != 4 && o.bits != 8 && o.bits != 16 && o.bits != 32)
    return fail(NWK_EINVAL, "nwk_ctx_create: bits must be 0/4/8/16/32");
  if (ndev <= 0) return fail(NWK_EDEVICE, "nwk_ctx_create: no HIP device visible");
  if (o.device < 0 || o.device >= ndev) return fail(NWK_EINVAL, "nwk_ctx_create: device %d of %d", o.device, ndev);
  std::unique_ptr<nwk_ctx> c(new nwk_ctx);
  c->opts = o;
  c->device = o.device;
  HIP_TRY(hipSetDevice(c->device));
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, c->device));
  c->cus = prop.multiProcessorCount;
  // NWK_CU_RESERVE=r (experiment, tools/overlap_probe.py): the engine's stream
  // runs on all but r CUs (a CU mask), and the persistent grids are sized for
  // the rest, so a collective launched on another stream (RCCL's kernels need
  // 248-256 VGPRs and 37.7 KB of LDS per 256-thread block) finds room while a
  // fill launch holds every other CU's register file
  const int reserve = getenv("NWK_CU_RESERVE") ? atoi(getenv("NWK_CU_RESERVE")) : 0;
  if (reserve > 0 && reserve < c->cus) {
    std::vector<uint32_t> mask((size_t)(c->cus + 31) / 32, 0u);
    for (int q = 0; q < c->cus - reserve; ++q) mask[(size_t)q / 32] |= 1u << (q % 32);
    HIP_TRY(hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask.size(), mask.data()));
    c->cus -= reserve;
  } else {
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  }
  for (auto& e : c->ev) HIP_TRY(hipEventCreate(&e));
  size_t fr = 0, tot = 0;
  HIP_TRY(hipMemGetInfo(&fr, &tot));
  if (o.workspace_bytes > 0) {
    c->budget = o.workspace_bytes;
  } else {
    c->budget = (int64_t)((double)fr * 0.92) - (512ll << 20);
    if (c->budget < (64ll << 20)) c->budget = 64ll << 20;
  }
  unsigned hc = std::thread::hardware_concurrency();
  c->host_threads = o.host_threads > 0 ? o.host_threads : (int)std::min(16u, hc ? hc : 1u);
  HIP_TRY(c->d_ctl.ensure(256) == NWK_OK ? hipSuccess : hipErrorOutOfMemory);
  *out = c.release();
  return NWK_OK;
}

int nwk_set_sequences(nwk_ctx* c, const uint8_t* seqs, const int64_t* offsets, int32_t k) {
  if (!c || (k > 0 && (!seqs || !offsets)) || k < 0) return fail(NWK_EINVAL, "nwk_set_sequences: bad argument");
  for (int s = 0; s < k; ++s)
    if (offsets[s + 1] < offsets[s] || offsets[s + 1] - offsets[s] > (1 << 30))
      return fail(NWK_EINVAL, "nwk_set_sequences: bad offsets at %d", s);
  c->k = k;
  const int64_t base = k ? offsets[0] : 0;
  if (k) c->off.assign(offsets, offsets + k + 1);
  else c->off.assign(1, 0);
  const int64_t total = k ? offsets[k] - base : 0;
  if (total) c->seqs.assign(seqs + base, seqs + base + total);
  else c->seqs.clear();
  for (auto& v : c->off) v -= base;
  bool seen[256] = {};
  for (uint8_t b : c->seqs) seen[b] = true;
  c->alpha = 0;
  for (int b = 0; b < 256; ++b)
    if (seen[b]) c->code_of[b] = (uint8_t)c->alpha++;
  c->has_us = seen[(unsigned char)'_'];
  c->built[0] = c->built[1] = false;
  for (auto& b : c->built_sel) b = false;
  c->built_yw = false;
  // layout: codes 8-aligned; E / SEL with kEPad entries before column 0 and kETail past the end
  c->c_off.resize(k);
  c->e_off.resize(k);
  int64_t co = kCodesFrontPad, eo = 0;
  for (int s = 0; s < k; ++s) {
    const int64_t L = c->off[s + 1] - c->off[s];
    c->c_off[s] = co;
    co += round_up(L + 8, 8);
    c->e_off[s] = eo + kEPad;
    eo += kEPad + L + kETail;
  }
  return NWK_OK;
}

}  // extern "C"

namespace {

// Builds (once per sequence set and encoding) the device codes and the
// expanded column array E: E[a] packs the encodings of y[a..a+3].
// kind 0: profile codes (code*8 in E, code in codes); kind 1: raw bytes.
int build_encoding(nwk_ctx* c, int kind) {
  if (c->built[kind]) return NWK_OK;
  const int k = c->k;
  const int64_t ncodes =
      (k ? c->c_off[k - 1] + round_up(c->off[k] - c->off[k - 1] + 8, 8) : kCodesFrontPad) + kCodesTailPad;
  const int64_t nE = k ? c->e_off[k - 1] + (c->off[k] - c->off[k - 1]) + kETail : 64;
  std::vector<uint8_t> codes((size_t)ncodes, 0);
  std::vector<uint32_t> E((size_t)nE, 0);
  for (int s = 0; s < k; ++s) {
    const uint8_t* y = c->seqs.data() + c->off[s];
    const int64_t L = c->off[s + 1] - c->off[s];
    uint8_t* cd = codes.data() + c->c_off[s];
    for (int64_t a = 0; a < L; ++a) cd[a] = kind == 0 ? c->code_of[y[a]] : y[a];
    uint32_t* e = E.data() + c->e_off[s];
    for (int64_t a = -kEPad; a < L + kETail; ++a) {
      uint32_t v = 0;
      for (int q = 0; q < 4; ++q) {
        const int64_t t = a + q;
        uint32_t b = 0;
        if (t >= 0 && t < L) b = kind == 0 ? (uint32_t)c->code_of[y[t]] * 8u : y[t];
        v |= b << (8 * q);
      }
      e[a] = v;
    }
  }
  int rc;
  if ((rc = c->d_codes[kind].ensure(codes.size())) != NWK_OK) return rc;
  if ((rc = c->d_E[kind].ensure(E.size() * 4)) != NWK_OK) return rc;
  HIP_TRY(hipMemcpy(c->d_codes[kind].p, codes.data(), codes.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_E[kind].p, E.data(), E.size() * 4, hipMemcpyHostToDevice));
  c->built[kind] = true;
  return NWK_OK;
}

// kPacked selector stream (same indexing as E): SEL[a] = {code(y[a]), hi,
// 4 + code(y[a-1]), hi} -- the v_perm selector of the substitution profile
// bytes of a row pair at column a+1 (row q) and a (row q+4); hi = 0x0d
// (byte 0xff: both K < 0) or 0x0c (byte 0x00: both K >= 0) sign-extends.
// kPacked2 (lag 64): SEL64[a] = {code(y[a]), hi, 4 + code(y[a-64]), hi}.
int build_sel(nwk_ctx* c, int neg, int lag) {
  const int idx = neg + (lag == 64 ? 2 : 0);
  if (c->built_sel[idx]) return NWK_OK;
  const int k = c->k;
  const int64_t nE = k ? c->e_off[k - 1] + (c->off[k] - c->off[k - 1]) + kETail : 64;
  std::vector<uint32_t> S((size_t)nE, 0);
  const uint32_t hi = neg ? 0x0du : 0x0cu;
  for (int s = 0; s < k; ++s) {
    const uint8_t* y = c->seqs.data() + c->off[s];
    const int64_t L = c->off[s + 1] - c->off[s];
    uint32_t* e = S.data() + c->e_off[s];
    auto code = [&](int64_t t) -> uint32_t { return t >= 0 && t < L ? c->code_of[y[t]] : 0u; };
    for (int64_t a = -kEPad; a < L + kETail; ++a) e[a] = code(a) | hi << 8 | (4u + code(a - lag)) << 16 | hi << 24;
  }
  int rc;
  if ((rc = c->d_sel[idx].ensure(S.size() * 4)) != NWK_OK) return rc;
  HIP_TRY(hipMemcpy(c->d_sel[idx].p, S.data(), S.size() * 4, hipMemcpyHostToDevice));
  c->built_sel[idx] = true;
  return NWK_OK;
}

// kBits y windows: per position p (kYwFront before column 0 .. kYwTail past
// the end) two dwords, bit 31 - q of dword k = bit k of code(y[p + q]) (0
// outside the sequence).  nw_align_bits lane t reads position s_half - 32 t.
constexpr int64_t kYwFront = kBitsRows + 128, kYwTail = kBitsRows + 512;
int build_yw(nwk_ctx* c) {
  if (c->built_yw) return NWK_OK;
  const int k = c->k;
  c->yw_off.assign((size_t)k, 0);
  int64_t tot = 0;
  for (int s = 0; s < k; ++s) {
    c->yw_off[s] = tot + kYwFront;
    tot += kYwFront + (c->off[s + 1] - c->off[s]) + kYwTail;
  }
  std::vector<uint32_t> W((size_t)std::max<int64_t>(2 * tot, 2), 0);
  for (int s = 0; s < k; ++s) {
    const uint8_t* y = c->seqs.data() + c->off[s];
    const int64_t L = c->off[s + 1] - c->off[s];
    uint32_t* w = W.data() + 2 * (c->yw_off[s] - kYwFront);
    auto code = [&](int64_t t) -> uint32_t { return t >= 0 && t < L ? c->code_of[y[t]] : 0u; };
    uint32_t w0 = 0, w1 = 0;  // window of position p - 1
    for (int64_t q = 0; q < 31; ++q) {  // prime: positions p = -kYwFront - 1 .. covers y[p .. p+31]
      const uint32_t cd = code(-kYwFront - 1 + q);
      w0 = (w0 << 1) | (cd & 1u);
      w1 = (w1 << 1) | ((cd >> 1) & 1u);
    }
    for (int64_t p = -kYwFront; p < L + kYwTail; ++p) {
      const uint32_t cd = code(p + 31);  // the window's newest column enters at bit 0
      w0 = (w0 << 1) | (cd & 1u);
      w1 = (w1 << 1) | ((cd >> 1) & 1u);
      w[2 * (p + kYwFront)] = w0;
      w[2 * (p + kYwFront) + 1] = w1;
    }
  }
  int rc;
  if ((rc = c->d_yw.ensure(W.size() * 4)) != NWK_OK) return rc;
  HIP_TRY(hipMemcpy(c->d_yw.p, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  c->built_yw = true;
  return NWK_OK;
}

struct Plan {
  int mode, bits, kind;
  int K0, K1;
};

// Scoring of a call: the reference's linear gaps (pxy, pgap), or the
// build-defined affine variant (pxy, go, ge) of SURVEY §8 a9.
struct Scoring {
  int pxy, pgap;
  bool affine;
  int go, ge;
};

// nw_align_pka keeps H, E and F as 4 x (value - base) + tag + kPkaBias in int16
// halves.  H is (go + ge)-Lipschitz in the Manhattan distance (one gap step
// changes it by at most go + ge); a half's cells at one step lie
// within distance 640 of its base cell, re-centred every 64 steps, and E, F, the
// diagonal candidate sit at most 2(go + ge) + pxy above H.  So every value stays
// inside [0, 32000) when 4 (650 (go + ge) + pxy + 4) <= 15900 (bias 16000,
// +inf 32000, kernels:"Packed affine fill").  The profile bytes hold 4 pxy.
bool pka_admissible(const Scoring& sc) {
  if (sc.pxy < 0 || sc.go < 0 || sc.ge < 0 || 4 * (int64_t)sc.pxy > 255) return false;
  return 4 * (650 * ((int64_t)sc.go + sc.ge) + sc.pxy + 4) <= 15900;
}

int choose_plan(const nwk_ctx* c, const Scoring& sc, Plan* pl) {
  const int pxy = sc.pxy, pgap = sc.pgap;
  if (sc.affine) {
    // packed band pairs (nw_align_pka) where the int16 window provably holds
    // and the alphabet fits the 4-entry profile; opts.kernel = 1 (unpacked) or
    // NWK_AFFPK=0 keeps nw_align_affine
    static const int affpk_env = getenv("NWK_AFFPK") ? atoi(getenv("NWK_AFFPK")) : 1;
    const bool pk = c->opts.kernel != 1 && affpk_env != 0 && c->alpha <= 4 && pka_admissible(sc);
    pl->mode = pk ? kAffinePk : kAffine;
    // bit-sliced planes (nw_align_gotoh) where an instantiation exists for the
    // scoring (C5's 3/3/1, the linear 3/2 and 5/1 as go = 0, the tests') and the
    // alphabet fits two code planes; opts.kernel 7 asks for it, 1 keeps
    // nw_align_affine, 2 / 3 nw_align_pka; NWK_GOTOH=0 disables it under "auto"
    static const int gotoh_env = getenv("NWK_GOTOH") ? atoi(getenv("NWK_GOTOH")) : 1;
    const bool want_gotoh = c->opts.kernel == 7 || (c->opts.kernel == 0 && gotoh_env != 0);
    if (want_gotoh && gotoh_admissible(sc.pxy, sc.go, sc.ge, c->alpha)) pl->mode = kGotoh;
    pl->bits = 4;          // 4-bit traceback codes
    pl->kind = pk || pl->mode == kGotoh ? 0 : 1;  // profile codes / raw bytes (compare)
    pl->K0 = 0;
    pl->K1 = pxy;
    return NWK_OK;
  }
  if (pxy < 0 || pgap < 0) {
    pl->mode = kLiteral;
    pl->bits = 32;
  } else {
    const int64_t span = 2 * (int64_t)pgap + pxy;  // max |difference| the traceback compares
    int b = span < 16 ? 4 : span < 256 ? 8 : span < 65536 ? 16 : 32;
    if (c->opts.bits > b) b = c->opts.bits;
    pl->bits = b;
    const int64_t k0 = -2 * (int64_t)pgap, k1 = (int64_t)pxy - 2 * (int64_t)pgap;
    const bool bytes_ok = k0 >= -128 && k0 <= 127 && k1 >= -128 && k1 <= 127;
    pl->mode = (c->alpha <= 4 && bytes_ok) ? kProfile : kCompare;
  }
  pl->kind = pl->mode == kProfile ? 0 : 1;
  pl->K0 = (int)(-2 * (int64_t)pgap);
  pl->K1 = (int)((int64_t)pxy - 2 * (int64_t)pgap);
  // two cells per register when the profile bytes sign-extend uniformly
  // (K0, K1 both < 0 or both >= 0).  opts.kernel (or NWK_PACKED=0/1/2 when it is
  // 0) pins nw_align / nw_align_pk / nw_align_pk2 for tests and A/B runs; a
  // packed kernel asked for where it is not exact falls back to nw_align.
  static const int packed_env = getenv("NWK_PACKED") ? atoi(getenv("NWK_PACKED")) : 2;
  const int packed = c->opts.kernel > 0 && c->opts.kernel < 4 ? c->opts.kernel - 1 : packed_env;
  if (pl->mode == kProfile && pl->bits == 4 && packed > 0 && ((pl->K0 < 0) == (pl->K1 < 0)))
    pl->mode = packed == 1 ? kPacked : kPacked2;
  // bit-sliced difference planes (nw_align_bits) wherever they apply: pxy >= 0,
  // pgap in {1, 2}, <= 4 symbols.  opts.kernel 4 asks for it, 1..3 pin the
  // integer kernels, NWK_BITS_KERNEL=0 disables it under "auto" (A/B runs; the
  // driver's NWK_BITS is the storage width, opts.bits).
  // pl->bits keeps the profile kernels' width (the linear-space path uses it).
  static const int bits_env = getenv("NWK_BITS_KERNEL") ? atoi(getenv("NWK_BITS_KERNEL")) : 1;
  const bool want_bits = c->opts.kernel == 4 || c->opts.kernel == 5 || c->opts.kernel == 6 ||
                         (c->opts.kernel == 0 && bits_env != 0);
  if (want_bits && c->opts.bits == 0 && bits_admissible(pxy, pgap, c->alpha)) pl->mode = kBits;
  // bit-parallel columns (nw_align_col, same domain): opts.kernel 6 (under
  // "auto" use_col decides per job, once the pairs are known)
  if (pl->mode == kBits && c->opts.kernel == 6) pl->mode = kCol;
  return NWK_OK;
}

// 64-step super-blocks per band: the last band-row value of column n leaves
// lane 63 at step n + 62 (nw_align) or n + 126 (nw_align_pk, 2-column skew).
inline bool band_pairs(int mode) { return mode == kPacked2 || mode == kAffinePk; }
inline int sblocks_of(int mode, int64_t nch) { return (int)(nch + (mode == kPacked || band_pairs(mode) ? 2 : 1)); }
// Fill tasks per pair: bands, or band pairs (kPacked2, kAffinePk).
inline int64_t tasks_of(int mode, int64_t nb) { return mode == kBitsStrip ? 1 : band_pairs(mode) ? (nb + 1) / 2 : nb; }

// kPacked2 segmented traceback footprint for a speculative segment every E
// tasks (E = 0: one whole-pair segment): move buffers (segment k starts on
// row (k+1)*E*RT and may run to the border: capacity row + n) and control.
inline bool segmented(int mode) { return mode == kPacked || mode == kPacked2; }

void seg_footprint(PairWork* w, int mode, int E, int NG) {
  const int64_t RT = mode == kPacked2 ? 2 * kBandRows : kBandRows, nt = ceil_div(w->m, RT);
  if (w->n >= (1 << 22) || (int64_t)w->m + w->n >= (1 << 27)) E = 0;  // record fields: 22-bit column, 27-bit index
  if (E <= 0) NG = 1;
  while (NG > 1 && nt * NG > kMaxSegsPerPair) NG /= 2;     // 14-bit segment ids
  if (nt > kMaxSegsPerPair) E = 0, NG = 1;
  const int64_t K = E > 0 ? (nt - 1) / E : 0;
  w->spec = E;
  w->nguess = NG;
  w->njobs = K * (NG - 1);
  w->segops_b = round_up(NG * ((int64_t)E * RT * K * (K + 1) / 2 + K * (int64_t)w->n) + w->m + w->n, 16);
  w->segctl_b = nt * 4 + nt * NG * 32 + (w->m / 128 + 1) * 32 * 8 + w->njobs * 12;  // records: 32 slots per 128th row
}

// kBits geometry: 2048-row bands, 64 * (nchunks + 32) steps of 2 x 64 dwords,
// 2 NP <= 8 granules per 64-column chunk of each band's last row
inline int bits_sblocks(int64_t nch) { return (int)(nch + 32); }
constexpr int kBitsGranPerChunk = 8;

// kBits stored blocks per band: every block, or (bits_w > 0) the blocks of
// steps r + j with |j - i n / m| <= bits_w over the band's 2048 rows i
int64_t bits_nblk_of(int m, int n, int w) {
  const int64_t all = 8 * (int64_t)bits_sblocks(ceil_div(n, 64));
  if (w <= 0) return all;
  const int64_t width = (kBitsRows - 1) + ceil_div((int64_t)(kBitsRows - 1) * n, m) + 2 * (int64_t)w + 16;
  return std::min(all, ceil_div(width, 8) + 1);
}

// kCol geometry (nw_align_col, nwk_col.hip): lane t works on column s - t at
// step s; a band runs until lane 63 has column n - 1 and its last 32-column
// word of the band's last row is published (step 32 ceil(n / 32) + 94):
// 64 * (nchunks + 2) steps.  Stored blocks per band: every block, or (bits_w
// > 0) from bits_blk_lo(b) = (b 2048 n / m - w) / 8 on, covering every step
// c + t with |c - i n / m| <= w over the band's rows i (t < 64).
inline int col_sblocks(int64_t nch) { return (int)(nch + 2); }
int64_t col_nblk_of(int m, int n, int w) {
  const int64_t all = 8 * (int64_t)col_sblocks(ceil_div(n, 64));
  if (w <= 0) return all;
  const int64_t width = ceil_div((int64_t)(kBitsRows - 1) * n, m) + 2 * (int64_t)w + 64 + 16;
  return std::min(all, ceil_div(width, 8) + 1);
}

// kBitsStrip geometry (nw_align_strip, nwk_bits.hip): n' = columns per row
// pass, a multiple of 64 with >= 32 junk columns past n (the wrap's masked
// bits sit there); the strip runs until row m - 1 reaches column n - 1.
inline int strip_np(int n) { return (int)round_up((int64_t)n + 32, 64); }
inline int strip_sblocks(int m, int n) {
  const int np = strip_np(n), nb = (int)ceil_div(m, kBitsRows);
  const int64_t last = (int64_t)(nb - 1) * np + (n - 1) + (m - (int64_t)kBitsRows * (nb - 1) - 1);
  return (int)(last / 64 + 1);
}
// LDS hand-off ring per wave (dwords): one 64-column chunk of a pass's last row
// per slot, 2 NP packed dwords each; at most kStripMaxChunks chunks keeps 4
// workgroups (16 waves) per CU; at least 64 chunks keeps the hand-off's lag
// (n' / 64 - 32 super-blocks) and the lanes' 32-super-block pass entry apart
constexpr int kStripMinChunks = 64;
inline int strip_max_chunks(int pgap) { return pgap == 1 ? 500 : 200; }
inline bool strip_admissible(int m, int n, int pgap) {
  const int nch = strip_np(n) / 64;
  return m > 0 && n > 0 && nch >= kStripMinChunks && nch <= strip_max_chunks(pgap);
}
// stored 8-step blocks: full (the whole strip) or, windowed, per band; the
// bands' windows must not overlap (a block is stored into one window only) --
// a pair whose windows would overlap keeps full storage
void strip_storage(PairWork* w) {
  const int np = strip_np(w->n), nb = (int)ceil_div(w->m, kBitsRows);
  const int64_t full = 8 * (int64_t)strip_sblocks(w->m, w->n);
  if (w->bits_w > 0) {
    const int64_t width = (kBitsRows - 1) + ceil_div((int64_t)(kBitsRows - 1) * w->n, w->m) + 2 * (int64_t)w->bits_w + 16;
    const int64_t nblk = ceil_div(width, 8) + 1;
    bool ok = nb * nblk < full;
    for (int k = 0; ok && k + 1 < nb; ++k)
      ok = strip_blk_lo(k + 1, w->m, w->n, np, w->bits_w) >= strip_blk_lo(k, w->m, w->n, np, w->bits_w) + nblk;
    if (ok) {
      w->bits_nblk = (int)nblk;
      w->mat_dw = nb * nblk * 1024;
      return;
    }
    w->bits_w = 0;
  }
  w->bits_nblk = (int)full;
  w->mat_dw = full * 1024;
}

// kAffinePk stored super-blocks per band pair (bits_w > 0): pka_sb_lo(p) lies
// at or below the steps of its rows' window cells (>= R n / m - w - 1) and the
// highest is below (R + 1024) n / m + w + 127 (lane 63, the odd band's skew)
int64_t pka_nsb_of(int m, int n, int w) {
  const int64_t all = sblocks_of(kAffinePk, ceil_div(n, 64));
  if (w <= 0) return all;
  return std::min(all, ceil_div(ceil_div((int64_t)2 * kBandRows * n, m) + 2 * (int64_t)w + 256, 64) + 2);
}

// Storage window W of a job whose full matrices exceed the budget (see
// align_work).  kBits: the widest candidate whose whole job fits `batches`
// batches (1 unless NWK_WIN_BATCHES), at least 1024.  kAffinePk: 8192
// outright -- its paths stray up to ~4.6k columns (profiles/r02/pathdev_c5.txt)
// and it needs many rounds of band-pair tasks per batch anyway.  need(W) is
// the job's bytes at window W.  (Compares need / batches against the budget:
// batches x budget overflowed int64 for large budgets.)
template <class Need>
int choose_window(int mode, int batches, int64_t budget, Need&& need) {
  if ((mode == kAffinePk || mode == kGotoh) && batches <= 0) return 8192;
  const int64_t nb = batches > 0 ? batches : 1;
  static const int cand[] = {8192, 6144, 4096, 3072, 2560, 2048, 1536, 1024};
  for (int wc : cand)
    if (ceil_div(need(wc), nb) <= budget) return wc;
  return 1024;
}

// kGotoh stored 4-step blocks per band: every block of the band's steps
// 0 .. 32 (n / 32 + 65) - 1, or (bits_w > 0) from gotoh_blk_lo(b) on, the
// steps j + r of its cells (R0 + 1 + r, j), |j - i n / m| <= w, r < 2048
int64_t gotoh_nblk_of(int m, int n, int w) {
  const int64_t all = 8 * ((int64_t)(n >> 5) + 65);
  if (w <= 0) return all;
  return std::min(all, ceil_div(2 * (int64_t)w + ceil_div((int64_t)kBitsRows * n, m) + 2052, 4) + 1);
}

// gran: kGotoh granules per 32-column chunk of a band's last row (gotoh_granules)
void footprint(PairWork* w, int bits, int mode, bool affine, int gran = 0) {
  if (mode == kGotoh) {
    const int64_t nb = ceil_div(w->m, kBitsRows), nw = (w->n >> 5) + 1;
    w->segops_b = w->segctl_b = 0;
    w->spec = 0;
    w->bits_nblk = (int)gotoh_nblk_of(w->m, w->n, w->bits_w);
    w->mat_dw = nb * w->bits_nblk * 1024;
    w->bnd_gr = (nb - 1) * nw * gran;
    w->ops_b = round_up((int64_t)w->m + w->n, 256);  // (the walk writes whole 256-byte blocks)
    return;
  }
  if (mode == kBitsStrip) {
    w->segops_b = w->segctl_b = 0;
    w->spec = 0;
    strip_storage(w);
    w->bnd_gr = 0;  // the pass-to-pass hand-off stays in LDS
    // whole 128-byte lines per pair: the fused finalize's rows (op-region
    // layout) are written on one XCD and hashed on another, so no line may be
    // shared with a neighbour's rows (a stale copy in the hashing XCD's L2)
    w->ops_b = round_up((int64_t)w->m + w->n, 128);
    return;
  }
  if (mode == kCol) {
    const int64_t nb = ceil_div(w->m, kBitsRows), nw = ceil_div(w->n, 32);
    // segmented traceback (nwk_col.hip trace_col): a speculative segment per
    // band but the last -- move buffers in segops, records in d_segctl, info
    // in d_colinfo.  Off unless NWK_COL_SEG=1: a segment started on a band's
    // last row at the diagonal's column meets the pair's path only after
    // ~500-5000 rows on random sequences (tools/probe/segconv.c), so the pair
    // walk still crosses most of each band and then waits for the segment;
    // measured C4 99.1 vs 91.3 ms per step, big13 26.3 vs 25.9 (r4n).
    static const int seg_env = getenv("NWK_COL_SEG") ? atoi(getenv("NWK_COL_SEG")) : 0;
    const bool seg = seg_env != 0 && nb >= 2 && colseg_ok(w->n);
    w->spec = seg ? 1 : 0;
    w->nguess = 1;
    w->njobs = 0;
    w->segops_b = seg ? (nb - 1) * colseg_cap(w->n) : 0;
    w->segctl_b = seg ? (nb - 1) * ((int64_t)kBitsRows * 8 + 16) : 0;
    w->bits_nblk = (int)col_nblk_of(w->m, w->n, w->bits_w);
    w->mat_dw = nb * w->bits_nblk * 1024;
    w->bnd_gr = (nb - 1) * nw * 4;  // NP <= 4 granules per 32 columns of each band's last row
    w->ops_b = round_up((int64_t)w->m + w->n, 128);  // (whole lines per pair: the fused finalize's rows)
    return;
  }
  if (mode == kBits) {
    const int64_t nb = ceil_div(w->m, kBitsRows), nch = ceil_div(w->n, 64);
    w->segops_b = w->segctl_b = 0;
    w->spec = 0;
    w->bits_nblk = (int)bits_nblk_of(w->m, w->n, w->bits_w);
    w->mat_dw = nb * w->bits_nblk * 1024;
    w->bnd_gr = (nb - 1) * nch * kBitsGranPerChunk;
    w->ops_b = round_up((int64_t)w->m + w->n, 128);  // (whole lines per pair, as above)
    return;
  }
  const int64_t nb = ceil_div(w->m, kBandRows);
  const int64_t nch = ceil_div(w->n, 64);
  const int64_t nt = tasks_of(mode, nb);
  w->segops_b = w->segctl_b = 0;
  w->spec = 0;
  if (segmented(mode)) seg_footprint(w, mode, 0, 1);
  if (mode == kAffinePk && w->bits_w > 0) {
    w->bits_nblk = (int)pka_nsb_of(w->m, w->n, w->bits_w);
    w->mat_dw = 2 * nt * band_dwords(bits, w->bits_nblk);
  } else {
    w->mat_dw = (band_pairs(mode) ? 2 * nt : nb) * band_dwords(bits, sblocks_of(mode, nch));
  }
  w->bnd_gr = (nt - 1) * nch * 64 * (affine ? 2 : 1);  // affine: H and F boundary rows
  w->ops_b = round_up((int64_t)w->m + w->n, 16);
}

// Host finalize of one pair (skel:263-272 prefix, 135-157 trim/strings/hash;
// the penalty is the cost of the traced path, which telescopes to dp[m][n]).
struct Finalized {
  int32_t penalty;
  unsigned char hash[64];
};

void finalize_pair(const uint8_t* x, int m, const uint8_t* y, int n, const Scoring& sc,
                   const uint8_t* ops_rev, int nops, int ei, int ej, Finalized* out,
                   std::vector<uint8_t>* a1o = nullptr, std::vector<uint8_t>* a2o = nullptr) {
  const int64_t L0 = (int64_t)(ei > 0 ? ei : ej) + nops;
  std::vector<uint8_t> a1((size_t)L0), a2((size_t)L0);
  const int64_t pxy = sc.pxy;
  // linear: every gap column costs pgap; affine: a gap's first column costs
  // go + ge ('u'/'l' from the traceback, and the prefix run), the others ge
  const int64_t gopen = sc.affine ? (int64_t)sc.go + sc.ge : sc.pgap, gext = sc.affine ? sc.ge : sc.pgap;
  int64_t pen = 0;
  int64_t q = 0;
  if (ei > 0) {
    for (int t = 0; t < ei; ++t, ++q) { a1[q] = x[t]; a2[q] = '_'; }
    pen += gopen + (int64_t)(ei - 1) * gext;
  } else if (ej > 0) {
    for (int t = 0; t < ej; ++t, ++q) { a1[q] = '_'; a2[q] = y[t]; }
    pen += gopen + (int64_t)(ej - 1) * gext;
  }
  int i = ei, j = ej;
  for (int t = nops - 1; t >= 0; --t, ++q) {
    const uint8_t op = ops_rev[t];
    if (op == 'D') {
      a1[q] = x[i]; a2[q] = y[j];
      pen += x[i] == y[j] ? 0 : pxy;
      ++i; ++j;
    } else if (op == 'U' || op == 'u') {
      a1[q] = x[i]; a2[q] = '_';
      pen += op == 'u' ? gopen : gext;
      ++i;
    } else {
      a1[q] = '_'; a2[q] = y[j];
      pen += op == 'l' ? gopen : gext;
      ++j;
    }
  }
  (void)m; (void)n;
  // skel:137-144: keep what follows the last column that is '_' in both rows
  int64_t start = 0;
  for (int64_t t = L0 - 1; t >= 0; --t)
    if (a1[t] == '_' && a2[t] == '_') { start = t + 1; break; }
  const int64_t alen = L0 - start;
  char hx[256];
  if (alen >= (1 << 16)) {  // long rows (big13: ~125 KB, ~0.2 ms each): the two hashes on two threads
    std::thread t2([&]() { sha512_hex(a2.data() + start, (size_t)alen, hx + 128); });
    sha512_hex(a1.data() + start, (size_t)alen, hx);
    t2.join();
  } else {
    sha512_hex(a1.data() + start, (size_t)alen, hx);
    sha512_hex(a2.data() + start, (size_t)alen, hx + 128);
  }
  sha512_raw(hx, 256, out->hash);
  out->penalty = (int32_t)pen;
  if (a1o) a1o->assign(a1.begin() + start, a1.end());
  if (a2o) a2o->assign(a2.begin() + start, a2.end());
}

template <class F>
void parallel_for(int threads, int64_t n, F&& f) {
  if (n <= 0) return;
  if (threads <= 1 || n == 1) {
    for (int64_t t = 0; t < n; ++t) f(t);
    return;
  }
  std::atomic<int64_t> next{0};
  std::vector<std::thread> th;
  const int T = (int)std::min<int64_t>(threads, n);
  for (int w = 0; w < T; ++w)
    th.emplace_back([&]() {
      for (;;) {
        const int64_t t = next.fetch_add(1);
        if (t >= n) break;
        f(t);
      }
    });
  for (auto& t : th) t.join();
}

// Core: aligns `work` (any order) and writes penalties/hashes at work[].out.
// If strings != nullptr (single-pair API), also returns the alignment rows.
// The answer-hash chain of skel:159 advanced while later batches still run:
// results are marked ready by output index (= canonical pair id for a full
// call) and the chain consumes the ready prefix.
// caller index q's final result is in place (nwk_align_pairs_poll)
inline void mark_ready(nwk_ctx* c, int64_t q) {
  if (c->ready_out) c->ready_out[q].store(1, std::memory_order_release);
}

// Fused finalize: the host side of one batch's streamed records (see the
// consumer in align_work).  done: 0 running, 1 kernel finished (skip holds
// the window re-runs), 2 abandoned (an error path left align_work).
struct FusedSync {
  std::atomic<int> done{0};
  std::vector<char> skip;
  int64_t missing = 0;
};

// Fill-vs-walk guard (skel:274: the reference's penalty IS the fill's
// dp[m][n]).  The fill kernels below give their H(m, n) per pair
// (FillArgs::endv); every finalize compares it with the cost of the walked
// path, which equals it for a correct walk (the path telescopes to dp[m][n])
// and exceeds it when the walk read a wrong code.  A pair that disagrees is
// never published: it re-runs with full storage, and a second disagreement
// fails the call with NWK_EKERNEL.
bool guard_mode(int mode) {
  return mode == kCol || mode == kBits || mode == kGotoh || mode == kAffinePk || mode == kAffine || mode == kPacked ||
         mode == kPacked2 ||
         mode == kProfile || mode == kCompare || mode == kLiteral;
}

struct GuardLog {
  struct Bad {
    int64_t idx;  // dp index
    int endv, cost;
  };
  std::mutex mu;
  std::vector<Bad> bad;
  void add(int64_t idx, int endv, int cost) {
    std::lock_guard<std::mutex> g(mu);
    bad.push_back({idx, endv, cost});
  }
  std::vector<Bad> take() {
    std::lock_guard<std::mutex> g(mu);
    std::vector<Bad> r;
    r.swap(bad);
    return r;
  }
};

// A pair whose walk disagreed with its fill (cost INT_MIN: computed on the
// device, not copied back).  A path never costs less than the DP minimum, so
// a cost below H(m, n) convicts the fill; above it, the walk read a wrong code
// (or the fill's minimum is too low).
int guard_rerun(const nwk_ctx* c, PairWork* w, int endv, int cost, nwk_stats* st) {
  const char* who = cost == INT_MIN ? "the walk or the fill"
                    : cost < endv   ? "the fill (a valid path costs less than its H(m, n))"
                                    : "the walk (a wrong code read), or the fill";
  if (w->guard >= 1)
    return fail(NWK_EKERNEL, "pair %lld (%d x %d): the walked path's cost %d differs from the fill's H(m, n) = %d "
                "again after a full-storage re-run: %s is wrong", (long long)w->id, w->m, w->n, cost, endv, who);
  if (c->opts.verbose || getenv("NWK_GUARD_LOG"))
    fprintf(stderr, "nwk guard: pair %lld (%d x %d, window %d): walked path cost %d, fill H(m, n) %d -> %s; re-run "
            "with full storage\n", (long long)w->id, w->m, w->n, w->bits_w, cost, endv, who);
  w->guard += 1;
  st->guard_reruns += 1;
  return NWK_OK;
}

struct Chain {
  const uint8_t* hashes = nullptr;  // [P][64] raw problem hashes
  std::vector<char> ready;
  std::vector<uint64_t> kw;         // [P][80] second-block schedules (prepare), off the chain's critical path
  std::vector<char> has_kw;
  int64_t next = 0;
  ChainAcc acc;  // acc starts as "" (skel:121)
  void init(const uint8_t* h, int64_t P) {
    hashes = h;
    ready.assign((size_t)P, 0);
    kw.assign((size_t)P * 80, 0);
    has_kw.assign((size_t)P, 0);
  }
  // pair p's schedule (any thread, once its hash is written, before it is marked ready)
  void prepare(int64_t p) {
    chain_schedule(hashes + 64 * p, kw.data() + 80 * p);
    has_kw[p] = 1;
  }
  void advance() {
    const int64_t P = (int64_t)ready.size();
    while (next < P && ready[next]) {
      if (!has_kw[next]) prepare(next);
      chain_step(&acc, kw.data() + 80 * next);
      ++next;
    }
  }
  // hash_hex[129]: the answer ("" for no pairs)
  void hex(char* out) const {
    chain_hex(acc, out);
    out[acc.empty ? 0 : 128] = 0;
  }
};

// Linear-space traceback for pairs whose DP matrix does not
// fit the HBM budget (or for every pair when opts.linear_space = G > 0).
// Pass 1 fills all bands keeping only their boundary rows (the granules,
// m/512 x n x 8 B).  Then, from the bottom up, a group of G bands plus the
// band above it (whose last row the trace reads) is recomputed -- all bands of
// the group at once, each from the stored boundary row above it -- into a
// scratch matrix of G + 1 bands, and the trace walks through the group to its
// top row.  Same kernel (nw_align, plain layout) and tie-breaks as the stored
// path, so the results are identical; the price is a second fill.  The pairs
// of a batch share every launch: pass 1 is one launch, and each round
// recomputes and traces the current group of every pair still tracing.
struct LinGeo {
  int nb, nch, sbl, G, ngroups;
  int64_t bdw, bnd_gr, scratch_dw, ops_cap, bytes;
};

LinGeo lin_geo(const Plan& pl, const PairWork& w, int G) {
  LinGeo g;
  g.nb = (int)ceil_div(w.m, kBandRows);
  g.nch = (int)ceil_div(w.n, 64);
  g.sbl = sblocks_of(pl.mode, g.nch);
  g.bdw = band_dwords(pl.bits, g.sbl);
  g.G = std::max(1, std::min(G, g.nb));
  g.ngroups = (int)ceil_div(g.nb, g.G);
  g.bnd_gr = (int64_t)std::max(1, g.nb - 1) * g.nch * 64;
  g.scratch_dw = (int64_t)(g.G + 1) * g.bdw;
  g.ops_cap = round_up((int64_t)w.m + w.n + 16 * (g.ngroups + 1), 16);
  g.bytes = g.bnd_gr * 8 + g.scratch_dw * 4 + g.ops_cap + 1024;
  return g;
}

Plan lin_plan(const Plan& pl0) {
  Plan pl = pl0;
  if (pl.mode == kPacked || pl.mode == kPacked2 || pl.mode == kBits || pl.mode == kBitsStrip || pl.mode == kCol)
    pl.mode = kProfile;  // same bits, codes, K0/K1
  return pl;
}

// G for one pair alone in the budget (0 if even two bands do not fit)
int lin_auto_groups(const nwk_ctx* c, const Plan& pl, const PairWork& w) {
  const LinGeo g = lin_geo(pl, w, 1);
  const int64_t avail = c->budget - g.bnd_gr * 8 - 2 * ((int64_t)w.m + w.n) - (1ll << 20);
  const int64_t G = avail / (g.bdw * 4) - 1;
  return G < 1 ? 0 : (int)std::min<int64_t>(G, g.nb);
}

int align_linear_batch(nwk_ctx* c, const Plan& pl0, const Scoring& sc, const PairWork* ws, int np, int G,
                       Finalized* outs, std::vector<uint8_t>* a1, std::vector<uint8_t>* a2, nwk_stats* st) {
  const Plan pl = lin_plan(pl0);
  int rc;
  std::vector<LinGeo> geo((size_t)np);
  std::vector<PairDesc> pd((size_t)np);
  std::vector<int64_t> scr_off((size_t)np), ops_off((size_t)np);
  int64_t bnd = 0, scr = 0, ops = 0, ntasks = 0;
  for (int q = 0; q < np; ++q) {
    const PairWork& w = ws[q];
    const LinGeo& g = geo[q] = lin_geo(pl, w, G);
    PairDesc& d = pd[q];
    memset(&d, 0, sizeof d);
    d.x_off = c->c_off[w.i];
    d.y_off = c->c_off[w.j];
    d.e_off = c->e_off[w.j];
    d.bnd_off = bnd;
    d.m = w.m;
    d.n = w.n;
    d.nbands = g.nb;
    d.nchunks = g.nch;
    d.sblocks = g.sbl;
    d.slot = q;
    scr_off[q] = scr;
    ops_off[q] = ops;
    bnd += g.bnd_gr;
    scr += g.scratch_dw;
    ops += g.ops_cap;
    ntasks += g.nb;
  }
  const int64_t bnd_need_b = bnd * 8 + 4096;
  const int64_t scratch_b0 = round_up(bnd_need_b, 256);
  const int64_t ops_base_b = scratch_b0 + round_up(scr * 4, 256);
  const int64_t work_b = ops_base_b + ops + 4096;
  void* const old_work = c->d_work.p;
  if ((rc = c->d_work.ensure((size_t)work_b)) != NWK_OK) return rc;
  if (c->d_work.p != old_work) c->clean_b = 0;
  static const int lin_zero = getenv("NWK_LIN_ZERO") ? atoi(getenv("NWK_LIN_ZERO")) : 0;  // debug A/B
  if (lin_zero == 1) c->clean_b = 0;
  if (lin_zero == 2) HIP_TRY(hipMemsetAsync(c->d_work.p, 0, (size_t)work_b, c->stream));
  if (bnd_need_b > c->clean_b)
    HIP_TRY(hipMemsetAsync(c->d_work.as<uint8_t>() + c->clean_b, 0, (size_t)(bnd_need_b - c->clean_b), c->stream));
  c->clean_b = bnd_need_b;
  if ((rc = c->d_pairs.ensure(sizeof(PairDesc) * np)) != NWK_OK) return rc;
  if ((rc = c->d_tasks.ensure(sizeof(int2) * ntasks)) != NWK_OK) return rc;
  if ((rc = c->d_oplen.ensure(sizeof(int) * np)) != NWK_OK) return rc;
  if ((rc = c->d_endij.ensure(sizeof(int2) * np)) != NWK_OK) return rc;
  if ((rc = c->d_done.ensure(sizeof(unsigned) * np)) != NWK_OK) return rc;
  for (int q = 0; q < np; ++q) pd[q].mat_off = scratch_b0 / 4 + scr_off[q];
  if (c->opts.verbose >= 3) {
    fprintf(stderr, "nwk linear batch: %d pairs, G %d, budget %lld, work %lld B at %p, clean %lld; ids", np, G,
            (long long)c->budget, (long long)work_b, c->d_work.p, (long long)c->clean_b);
    for (int q = 0; q < np; ++q) fprintf(stderr, " %lld", (long long)ws[q].id);
    fprintf(stderr, "\n");
  }
  FillArgs fa{};
  memset(&fa, 0, sizeof fa);
  fa.pairs = c->d_pairs.as<PairDesc>();
  fa.tasks = c->d_tasks.as<int2>();
  fa.codes = c->d_codes[pl.kind].as<uint8_t>();
  fa.E = c->d_E[pl.kind].as<uint32_t>();
  fa.mat = c->d_work.as<uint32_t>();
  fa.bnd = c->d_work.as<unsigned long long>();
  fa.counter = c->d_ctl.as<unsigned>();
  fa.err = c->d_ctl.as<unsigned>() + 16;
  fa.done = c->d_done.as<unsigned>();
  fa.ops = c->d_work.as<uint8_t>();
  fa.oplen = c->d_oplen.as<int>();
  fa.endij = c->d_endij.as<int2>();
  fa.epoch = ++c->epoch;  // the group passes read pass 1's boundary rows under the same epoch
  if (fa.epoch == 0) fa.epoch = ++c->epoch;
  fa.K0 = pl.K0;
  fa.K1 = pl.K1;
  fa.ntasks_pairs = np;
  const int grid = fill_blocks_per_cu(pl.mode, pl.bits) * c->cus;
  std::vector<int2> tk;
  tk.reserve((size_t)ntasks);
  std::vector<int> ol((size_t)np, 0);
  std::vector<int2> ej((size_t)np);
  // one launch over the tasks in tk, waited for
  auto launch = [&](int mode, double* ms_acc) -> int {
    const int64_t nt = (int64_t)tk.size();
    HIP_TRY(hipMemcpyAsync(c->d_pairs.p, pd.data(), sizeof(PairDesc) * np, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_tasks.p, tk.data(), sizeof(int2) * nt, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_ctl.p, 0, 256, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_done.p, 0, sizeof(unsigned) * np, c->stream));
    fa.ntasks = (int)nt;
    fa.lin_mode = mode;
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(launch_fill(pl.mode, pl.bits, fa, (int)std::min<int64_t>(grid, ceil_div(nt, 4)), c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    unsigned herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, fa.err, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(ol.data(), fa.oplen, 4 * (size_t)np, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(ej.data(), fa.endij, 8 * (size_t)np, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (herr) return fail(NWK_EKERNEL, "linear-space pass %d of a %d-pair batch failed (err=%u)", mode, np, herr);
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[1]));
    *ms_acc += ms;
    st->fill_launches += 1;
    return NWK_OK;
  };
  for (int q = 0; q < np; ++q)
    for (int b = 0; b < geo[q].nb; ++b) tk.push_back(make_int2(q, b));
  // fill-vs-walk guard: pass 1 fills every cell and gives each pair's H(m, n)
  static const int guard_env = getenv("NWK_GUARD") ? atoi(getenv("NWK_GUARD")) : 1;
  std::vector<int> endv((size_t)np, 0);
  if (guard_env != 0) {
    if ((rc = c->d_endv.ensure(sizeof(int) * np)) != NWK_OK) return rc;
    HIP_TRY(hipMemsetAsync(c->d_endv.p, 0, sizeof(int) * np, c->stream));
    fa.endv = c->d_endv.as<int>();
    fa.pgap = sc.pgap;
  }
  if ((rc = launch(1, &st->fill_ms)) != NWK_OK) return rc;
  if (guard_env != 0) {
    HIP_TRY(hipMemcpy(endv.data(), fa.endv, sizeof(int) * np, hipMemcpyDeviceToHost));
    st->guard_checked += np;
  }
  std::vector<int> ci((size_t)np), cj((size_t)np);
  std::vector<int64_t> off((size_t)np, 0);
  std::vector<std::vector<std::pair<int64_t, int>>> pieces((size_t)np);
  for (int q = 0; q < np; ++q) ci[q] = ws[q].m, cj[q] = ws[q].n;
  for (;;) {
    tk.clear();
    std::vector<int> act;
    for (int q = 0; q < np; ++q) {
      if (ci[q] <= 0 || cj[q] <= 0) continue;
      const LinGeo& g = geo[q];
      const int gb1 = (ci[q] - 1) / kBandRows;
      const int b0 = std::max(0, gb1 - g.G + 1);
      const int gb0 = std::max(0, b0 - 1);
      PairDesc& d = pd[q];
      d.mat_off = scratch_b0 / 4 + scr_off[q] - (int64_t)gb0 * g.bdw;  // band b at scratch + (b - gb0) bands
      d.ops_off = ops_base_b + ops_off[q] + off[q];
      d.lin_nb = gb1 - gb0 + 1;
      d.lin_i = ci[q];
      d.lin_j = cj[q];
      d.lin_stop = b0 * kBandRows;
      for (int b = gb0; b <= gb1; ++b) tk.push_back(make_int2(q, b));
      act.push_back(q);
    }
    if (act.empty()) break;
    if ((rc = launch(2, &st->traceback_ms)) != NWK_OK) return rc;
    for (int q : act) {
      if (ol[q] < 0 || off[q] + ol[q] > geo[q].ops_cap || ej[q].x > ci[q] || ej[q].y > cj[q] ||
          (ej[q].x == ci[q] && ej[q].y == cj[q]))
        return fail(NWK_EKERNEL, "linear-space trace of pair (%d x %d) stalled at (%d, %d)", ws[q].m, ws[q].n, ci[q], cj[q]);
      pieces[q].emplace_back(off[q], ol[q]);
      off[q] += round_up(ol[q], 16);
      ci[q] = ej[q].x;
      cj[q] = ej[q].y;
    }
  }
  std::vector<uint8_t> buf((size_t)std::max<int64_t>(ops, 1));
  HIP_TRY(hipMemcpy(buf.data(), c->d_work.as<uint8_t>() + ops_base_b, (size_t)ops, hipMemcpyDeviceToHost));
  parallel_for(a1 ? 1 : c->host_threads, np, [&](int64_t q) {
    std::vector<uint8_t> rev;
    rev.reserve((size_t)ws[q].m + ws[q].n);
    const uint8_t* base = buf.data() + ops_off[q];
    for (const auto& pc : pieces[q]) rev.insert(rev.end(), base + pc.first, base + pc.first + pc.second);
    finalize_pair(c->seqs.data() + c->off[ws[q].i], ws[q].m, c->seqs.data() + c->off[ws[q].j], ws[q].n, sc, rev.data(),
                  (int)rev.size(), ci[q], cj[q], &outs[q], a1, a2);
  });
  // the linear-space walk recomputes its bands from the same boundary rows, so
  // a re-run would repeat a disagreement: it fails the call
  if (guard_env != 0)
    for (int q = 0; q < np; ++q)
      if (outs[q].penalty != endv[q])
        return fail(NWK_EKERNEL, "linear-space pair %lld (%d x %d): the walked path costs %d but the fill's H(m, n) is %d",
                    (long long)ws[q].id, ws[q].m, ws[q].n, outs[q].penalty, endv[q]);
  for (int q = 0; q < np; ++q) st->matrix_bytes += geo[q].scratch_dw * 4;
  st->linear_space_pairs += np;
  st->batches += 1;
  return NWK_OK;
}

// Strips or band tasks for a kBits job (nw_align_strip vs nw_align_bits).  A
// strip sweeps all of a pair's bands in one wave: fewer steps (the 2047-step
// skew once per pair, not per band: ~16% on 8k pairs) and no inter-wave
// hand-off, but the pair's latency is its whole strip.  Estimated makespans
// in wave-steps: band tasks max(total band steps / slots, the longest pair's
// pipeline n + nb x 2112); strips the LPT list schedule of the strip lengths
// over the wave slots.  force: 1 = strips wherever admissible (tests).
bool use_strips(const nwk_ctx* c, const std::vector<PairWork>& work, int pgap, bool force, int* ring_out) {
  int ring = 0;
  int64_t npairs = 0;
  for (const auto& w : work) {
    if (w.m == 0 || w.n == 0) continue;
    if (!strip_admissible(w.m, w.n, pgap)) return false;
    ring = std::max(ring, strip_np(w.n) / 64 * 4 * pgap);
    ++npairs;
  }
  *ring_out = ring;
  if (npairs == 0) return false;
  if (force) return true;
  const int64_t slots_b = 4LL * bits_blocks_per_cu(pgap) * c->cus;
  const int64_t slots_s = 4LL * strip_blocks_per_cu(pgap, ring) * c->cus;
  double band_steps = 0, span = 0;
  std::vector<int64_t> len;
  len.reserve((size_t)npairs);
  for (const auto& w : work) {
    if (w.m == 0 || w.n == 0) continue;
    const int64_t nb = ceil_div(w.m, kBitsRows), nch = ceil_div(w.n, 64);
    band_steps += (double)nb * (nch + 32) * 64;
    span = std::max(span, (double)w.n + nb * (kBitsRows + 64.0));
    len.push_back(64LL * strip_sblocks(w.m, w.n));
  }
  const double est_b = std::max(band_steps / (double)slots_b, span);
  std::sort(len.begin(), len.end(), std::greater<int64_t>());
  std::vector<int64_t> heap((size_t)std::min<int64_t>(slots_s, npairs), 0);  // min-heap of slot finish times
  for (int64_t L : len) {
    std::pop_heap(heap.begin(), heap.end(), std::greater<int64_t>());
    heap.back() += L;
    std::push_heap(heap.begin(), heap.end(), std::greater<int64_t>());
  }
  const double est_s = (double)*std::max_element(heap.begin(), heap.end());
  // Beyond two rounds of strips per wave slot the band tasks keep every slot
  // busy too, and a strip step costs more than a band step (pass switches,
  // per-lane storage window): C4 on one GPU (8 rounds) fills in 86.8 ms as
  // bands vs 88.7 ms as strips, 100.9 vs 104.8 ms per step; a C4 shard of 8
  // ranks (1 round) stays on strips (14.5 vs 21.7 ms).
  if (npairs > 2 * slots_s) return est_s < 0.8 * est_b;
  return est_s < 0.95 * est_b;
}

int align_work(nwk_ctx* c, std::vector<PairWork>& work, const Scoring& sc, int32_t* penalties,
               uint8_t* hashes, std::vector<uint8_t>* a1, std::vector<uint8_t>* a2, Chain* chain = nullptr) {
  const double t_start = now_ms();
  nwk_stats st{};
  Plan pl;
  choose_plan(c, sc, &pl);
  if (sc.affine) {
    if (sc.pxy < 0 || sc.go < 0 || sc.ge < 0)
      return fail(NWK_EINVAL, "affine gaps need pxy, go, ge >= 0 (got %d, %d, %d)", sc.pxy, sc.go, sc.ge);
    // H values stay below the kernel's +inf (2^30 - 1) with room for one step
    for (const auto& w : work)
      if (((int64_t)w.m + w.n + 2) * ((int64_t)sc.go + sc.ge + sc.pxy) >= (1ll << 29))
        return fail(NWK_EINVAL, "affine scores of pair (%d x %d) would exceed the int32 range", w.m, w.n);
  }
  // Small jobs (e.g. one rank's shard of a multi-GPU run): band-pair tasks
  // (1024 rows, 16 cells per lane-step) too few to occupy the wave slots make
  // each pair's row sweep the critical path -- single bands (nw_align_pk,
  // 8 cells per lane-step) sweep a row in about half the time.
  if (pl.mode == kPacked2 && !getenv("NWK_PACKED") && c->opts.kernel == 0) {
    int64_t t2 = 0;
    for (const auto& w : work)
      if (w.m > 0 && w.n > 0) t2 += ceil_div(w.m, 2 * kBandRows);
    if (t2 < 8 * (int64_t)c->cus) pl.mode = kPacked;  // (2048 on 256 CUs; the kernels tie near there)
  }
  // nw_align_bits as rolling strips (kBitsStrip): NWK_STRIP / opts.kernel 5
  // force them (1) or band tasks (0); by default use_strips decides
  int strip_ring = 0;
  if (pl.mode == kBits) {
    static const int strip_env = getenv("NWK_STRIP") ? atoi(getenv("NWK_STRIP")) : -1;
    const int want = c->opts.kernel == 5 ? 1 : c->opts.kernel == 4 ? 0 : strip_env;
    if (want != 0 && use_strips(c, work, sc.pgap, want == 1, &strip_ring)) pl.mode = kBitsStrip;
  }
  // nw_align_col under "auto", wherever the bits kernels apply: a pair costs its
  // span n + ~100 per band there against n + 2112 per band for nw_align_bits,
  // its stores are windowed (write-bound jobs), its plain launches run 5
  // waves/SIMD and its pairs stream to the host finalize during the launch.
  // big13 24.1 vs 33 ms per step, C4 85 vs 100 ms, C3's 8 / 4 / 2-rank shards
  // 30 / 47 / 83 vs 47 / 61 / 97 ms, and since round 5 C3 on one GPU too
  // (155.2 vs 160.9 ms per step, profiles/r05/ab/c3_col_vs_bits.txt; round 4 at
  // 4 waves/SIMD and a device finalize after the launch: 160 vs 153 ms).
  // NWK_COL=0 keeps nw_align_bits (A/B runs), NWK_STRIP=1 forces strips.
  if ((pl.mode == kBits || pl.mode == kBitsStrip) && c->opts.kernel == 0) {
    static const int col_env = getenv("NWK_COL") ? atoi(getenv("NWK_COL")) : -1;
    static const bool strip_forced = getenv("NWK_STRIP") && atoi(getenv("NWK_STRIP")) == 1;
    const bool col = col_env == 1 || (col_env < 0 && !strip_forced);
    if (col) pl.mode = kCol;
  }
  const bool bitsy = pl.mode == kBits || pl.mode == kBitsStrip || pl.mode == kCol;
  bool gotoh = pl.mode == kGotoh;
  int ggran = gotoh ? gotoh_granules(sc.go, sc.ge) : 0;
  st.bits = bitsy ? 2 : pl.bits;
  st.mode = pl.mode;
  int rc;
  HIP_TRY(hipSetDevice(c->device));

  // Degenerate pairs (m == 0 or n == 0) have no DP cells: prefix only.
  // (capacity for one full-storage re-run of every pair: a kBits windowed pair
  // whose path leaves its window is appended once, and the async finalize
  // holds pointers into dp, so it must never reallocate)
  std::vector<PairWork> dp;
  dp.reserve(4 * work.size() + 16);
  for (auto& w : work) {
    st.cells += (double)w.m * (double)w.n;
    if (w.m == 0 || w.n == 0) {
      Finalized f;
      const uint8_t* x = c->seqs.data() + c->off[w.i];
      const uint8_t* y = c->seqs.data() + c->off[w.j];
      finalize_pair(x, w.m, y, w.n, sc, nullptr, 0, w.m, w.n, &f, a1, a2);
      penalties[w.out] = f.penalty;
      memcpy(hashes + 64 * w.out, f.hash, 64);
      if (chain) chain->ready[w.out] = 1;
      mark_ready(c, w.out);
    } else {
      footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
      dp.push_back(w);
    }
  }
  // nw_align_gotoh stores whole 2048-row bands plus their 2080-step skew, so a
  // short pair costs more than on the band-pair kernels: a pair that does not
  // fit the budget even at its 8192-column window runs the job on nw_align_pka
  // (or nw_align_affine) instead.
  if (gotoh) {
    bool fits = true;
    for (const auto& w : dp) {
      PairWork t = w;
      t.bits_w = 8192;
      footprint(&t, pl.bits, pl.mode, sc.affine, ggran);
      fits = fits && t.mat_dw * 4 + t.bnd_gr * 8 + 3 * t.ops_b + 8192 <= c->budget;
    }
    if (!fits) {
      const bool pk = c->alpha <= 4 && pka_admissible(sc);
      pl.mode = pk ? kAffinePk : kAffine;
      pl.kind = pk ? 0 : 1;
      st.mode = pl.mode;
      gotoh = false;
      ggran = 0;
      for (auto& w : dp) footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
    }
  }
  if (!dp.empty()) {
    if ((rc = build_encoding(c, pl.kind)) != NWK_OK) return rc;
    if ((bitsy || gotoh) && (rc = build_yw(c)) != NWK_OK) return rc;
    if ((pl.mode == kPacked || band_pairs(pl.mode)) &&
        (rc = build_sel(c, pl.K0 < 0 ? 1 : 0, band_pairs(pl.mode) ? 64 : 1)) != NWK_OK)
      return rc;
  }
  // kBits windowed storage.  When the job's full 2-bit matrices exceed the
  // workspace, store only the steps within W columns of each pair's diagonal
  // j = i n / m, W the widest candidate that fits the job in one batch (at
  // least 1024).  Paths of random C3 pairs stay within ~1.2k columns of it
  // (tools/pathdev.py); a path that leaves its window is detected by the
  // traceback and the pair re-runs with full storage (the retry list below),
  // so results never depend on W.  NWK_BITS_WIN: 0 off, W > 0 forced.
  //
  // kAffinePk (nw_align_pka) the same way, per 64-step super-block of a band
  // pair.  Its bands need many rounds of tasks per wave slot to run free of
  // the band-pair chains (a band pair dequeued right behind the one above
  // waits on it), which only a window gives at C5's size (full storage: 13
  // pairs per batch).  Affine paths stray further (C5 pairs: up to ~4.6k
  // columns, profiles/r02/pathdev_c5.txt), so it keeps W = 8192 and takes
  // more batches (C5: 4 of ~124 pairs, ~12 rounds of wave slots each).
  static const int win_env = getenv("NWK_BITS_WIN") ? atoi(getenv("NWK_BITS_WIN")) : -1;
  static const int winb_env = getenv("NWK_WIN_BATCHES") ? atoi(getenv("NWK_WIN_BATCHES")) : 0;
  if ((bitsy || pl.mode == kAffinePk || gotoh) && !dp.empty() && win_env != 0) {
    auto total_b = [&]() {
      int64_t mat = 0, bnd = 0, ops = 0;
      int64_t seg = 0;
      for (const auto& w : dp) mat += w.mat_dw, bnd += w.bnd_gr, ops += w.ops_b, seg += w.segops_b + w.segctl_b;
      return mat * 4 + bnd * 8 + 3 * ops + seg + 8192;
    };
    auto set_w = [&](int W) {
      for (auto& w : dp) {
        w.bits_w = W;
        footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
      }
    };
    int W = win_env > 0 ? win_env : 0;
    if (W == 0 && total_b() > c->budget)
      W = choose_window(pl.mode, winb_env, c->budget, [&](int wc) {
        set_w(wc);
        return total_b();
      });
    // Strips keep a 1024-column window even when full storage fits: below one
    // band's height a window writes only the lane words near the diagonal
    // (bits_lane_window), about half of them at 1024 -- C4's 8-rank shard
    // fits in full, and full storage wrote ~6 TB/s of HBM at 4 waves/SIMD.
    // Random 8k pairs' paths stay within ~400 columns (pathdev_c4.txt); a pair
    // whose path leaves re-runs in full.  NWK_STRIP_WIN overrides (0: full).
    static const int strip_win_env = getenv("NWK_STRIP_WIN") ? atoi(getenv("NWK_STRIP_WIN")) : 1024;
    if (W == 0 && pl.mode == kBitsStrip) W = strip_win_env;
    set_w(W);
    // nw_align_col stores 512 B per wave-step; at full storage a batch of many
    // concurrent bands writes faster than HBM takes it (C3's 8-rank shard and
    // big13 fit in full and wrote ~4-6 TB/s), so it keeps a window even when
    // full storage fits: per pair W = 2.5 x the paths' expected stray from the
    // diagonal, ~400 (n / 8000)^(2/3) columns for random sequences (max |dev|
    // over sampled pairs: 361 at C4's 8k, 1165 at C3's 50k,
    // profiles/r02/pathdev_*.txt), at least 1024 and at most a budget-forced W.
    // A path that strays further re-runs with full storage.  NWK_COL_WIN:
    // 0 = full storage when it fits, W > 0 forced.
    //
    // Only a job whose full storage would be written faster than ~4 TB/s takes
    // it: estimated fill time max(cells / 32k GCUPS, longest pair span x 0.3 us
    // per wave-step under load), span = n + 100 per band.  A job bound by one
    // long pair's span (big13: 94k steps) writes ~2.5 TB/s in full and keeps
    // full storage -- related sequences' paths stray far from the diagonal
    // (big13: 2.9k-50k columns, profiles/r04/pathdev_big13.txt), so a window
    // there sends nearly every pair to the re-run.
    static const int col_win_env = getenv("NWK_COL_WIN") ? atoi(getenv("NWK_COL_WIN")) : -1;
    bool col_wb = col_win_env > 0;
    if (pl.mode == kCol && col_win_env < 0) {
      double cells = 0, bytes = 0, span = 0;
      for (const auto& w : dp) {
        cells += (double)w.m * w.n;
        bytes += (double)w.m * w.n / 4;
        span = std::max(span, (double)w.n + 100.0 * (double)ceil_div(w.m, kBitsRows));
      }
      col_wb = bytes / std::max(cells / 3.2e13, span * 3.0e-7) > 4e12;
    }
    if (pl.mode == kCol && win_env < 0 && col_wb) {
      for (auto& w : dp) {
        const double est = 400.0 * std::pow(std::max(w.m, w.n) / 8000.0, 2.0 / 3.0);
        int wc = col_win_env > 0 ? col_win_env : (int)round_up(std::max<int64_t>(1024, (int64_t)(2.5 * est)), 256);
        if (W > 0) wc = std::min(wc, W);
        w.bits_w = wc;
        footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
      }
    }
  }
  st.window = dp.empty() ? 0 : dp[0].bits_w;
  // Largest first (LPT inside the device; longest bands dequeued first).
  // kPacked2 (NWK_SORT != 0): by traceback length m + n first, so the pairs
  // filled last -- whose traces form the kernel's tail -- are the shortest to trace.
  // NWK_SORT: 1 = m + n, 2 = max(m, n) (wide pairs merge their segments slowest), 0 = cells only
  static const int sort_trace = getenv("NWK_SORT") ? atoi(getenv("NWK_SORT")) : 2;
  const int by_trace = pl.mode == kPacked2 ? sort_trace : 0;
  std::sort(dp.begin(), dp.end(), [by_trace](const PairWork& a, const PairWork& b) {
    const int ka = by_trace == 1 ? a.m + a.n : std::max(a.m, a.n), kb = by_trace == 1 ? b.m + b.n : std::max(b.m, b.n);
    if (by_trace && ka != kb) return ka > kb;
    const double ca = (double)a.m * a.n, cb = (double)b.m * b.n;
    if (ca != cb) return ca > cb;
    return a.id < b.id;
  });
  // Segmented traceback (kPacked2): only the pairs dequeued last -- the last
  // NWK_SPEC_FRAC (default 0.35) of the cells -- trace speculatively (a
  // segment every NWK_SPEC tasks, default 2); earlier pairs' whole-pair
  // traces overlap the remaining fill anyway.
  if (segmented(pl.mode)) {
    // small jobs (nw_align_pk chosen above): every pair's trace is on the
    // critical path -> speculate everywhere with NWK_GUESS start columns per
    // boundary (default 8); large jobs: only the tail pairs
    const bool small = pl.mode == kPacked;
    static const int spec_env = getenv("NWK_SPEC") ? atoi(getenv("NWK_SPEC")) : 2;
    static const double frac_env = getenv("NWK_SPEC_FRAC") ? atof(getenv("NWK_SPEC_FRAC")) : -1.0;
    static const int guess_env = getenv("NWK_GUESS") ? atoi(getenv("NWK_GUESS")) : 0;
    const double frac = frac_env >= 0 ? frac_env : small ? 1.0 : 0.35;
    const int NG = guess_env > 0 ? guess_env : small ? 8 : 1;
    double tot = 0, acc = 0;
    for (const auto& w : dp) tot += (double)w.m * w.n;
    for (auto& w : dp) {
      const bool on = acc >= (1.0 - frac) * tot - 0.5;
      seg_footprint(&w, pl.mode, on ? std::max(0, spec_env) * (pl.mode == kPacked ? 2 : 1) : 0, NG);
      acc += (double)w.m * w.n;
    }
  }
  int bpc = pl.mode == kBits        ? bits_blocks_per_cu(sc.pgap)
            : pl.mode == kCol       ? col_blocks_per_cu(sc.pgap)
            : pl.mode == kBitsStrip ? strip_blocks_per_cu(sc.pgap, strip_ring)
                                    : fill_blocks_per_cu(pl.mode, pl.bits);
  // waves per SIMD: nw_align_pk2 measured best at 2 (band chains run at the
  // pace of their slowest member; more waves per SIMD only add waiting);
  // NWK_BPC overrides (experiments)
  if (pl.mode == kPacked2) bpc = std::min(bpc, 2);
  // nw_align_affine: 2 waves/SIMD beat 3 by ~4% kernel GCUPS on big13 and C5
  // (profiles/r01/ab_affine_bpc.json)
  if (pl.mode == kAffine) bpc = std::min(bpc, 2);
  if (pl.mode == kAffinePk) bpc = std::min(bpc, 2);
  if (gotoh) bpc = gotoh_blocks_per_cu(sc.pxy, sc.go, sc.ge);
  static const int bpc_cap = getenv("NWK_BPC") ? atoi(getenv("NWK_BPC")) : 0;
  if (bpc_cap > 0) bpc = std::min(bpc_cap, bitsy || gotoh ? bpc : fill_blocks_per_cu(pl.mode, pl.bits));
  const int grid = bpc * c->cus;
  float ms = 0;

  // at most one finalize in flight; joined on every exit path
  struct Joiner {
    std::thread t;
    void start(std::function<void()> f) { t = std::thread(std::move(f)); }
    void join() { if (t.joinable()) t.join(); }
    ~Joiner() { join(); }
  } fin;
  // Device finalize (nw_hash) when no input byte is '_' and the
  // batch has enough pairs for one lane per row to beat the host threads:
  // est. device ms ~ 0.007 per 128-byte block of the longest row (per wave
  // slot round), host ~ 350 bytes/us per thread.  NWK_DEVHASH=0/1 forces.
  static const int devhash_env = getenv("NWK_DEVHASH") ? atoi(getenv("NWK_DEVHASH")) : -1;
  const int fin_mode = c->opts.finalize == 1 ? 0 : c->opts.finalize >= 2 ? 1 : devhash_env;
  const bool dev_ok = a1 == nullptr && !c->has_us && fin_mode != 0;
  if (dev_ok && !dp.empty() && (rc = build_encoding(c, 1)) != NWK_OK) return rc;
  size_t pos = 0;
  // a pair re-runs in a later batch: with full storage (windowed storage whose
  // walk left the window, or a walk the fill-vs-walk guard rejected); the
  // affine path has no linear-space fallback, so there it takes the widest
  // doubled window that fits the budget when full storage does not
  auto requeue = [&](PairWork w) -> int {
    const int old_w = w.bits_w;
    w.bits_w = 0;
    footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
    auto need = [](const PairWork& x) {
      return x.mat_dw * 4 + x.bnd_gr * 8 + 3 * x.ops_b + x.segops_b + x.segctl_b + 8192;
    };
    if ((pl.mode == kAffinePk || gotoh) && need(w) > c->budget) {
      int nw = 0;
      for (int64_t cw = 2 * (int64_t)std::max(old_w, 1); cw < (1 << 30); cw *= 2) {
        PairWork t = w;
        t.bits_w = (int)cw;
        footprint(&t, pl.bits, pl.mode, sc.affine, ggran);
        if (need(t) > c->budget) break;
        nw = (int)cw;
        if (t.mat_dw >= w.mat_dw) break;  // as wide as full storage
      }
      if (nw == 0)
        return fail(NWK_ENOMEM, "pair %lld (%d x %d): its traceback left the %d-column storage window and "
                    "neither full storage (%lld B) nor a %d-column window fits the HBM budget %lld",
                    (long long)w.id, w.m, w.n, old_w, (long long)need(w), 2 * old_w, (long long)c->budget);
      w.bits_w = nw;
      footprint(&w, pl.bits, pl.mode, sc.affine, ggran);
    }
    if (dp.size() == dp.capacity())  // the async finalize holds pointers into dp
      return fail(NWK_ENOMEM, "pair %lld: too many re-runs", (long long)w.id);
    dp.push_back(w);
    return NWK_OK;
  };
  // fill-vs-walk guard mismatches found by the host finalize threads (dp index, H(m, n), path cost)
  GuardLog gl;
  static const int guard_env = getenv("NWK_GUARD") ? atoi(getenv("NWK_GUARD")) : 1;
  const bool guard_on = guard_env != 0;
  std::vector<std::shared_ptr<FusedSync>> fused_all;  // streamed batches (checked after the last join)
  double h_setup = 0, h_sync = 0, h_join = 0, h_last = 0;  // host phases (verbose)
  const bool lin_all = c->opts.linear_space > 0 && !sc.affine;  // (tests: every pair through f2)
  for (;;) {
  while (pos < dp.size()) {
    // ---- form a batch that fits the HBM budget
    size_t end = pos;
    bool lin_one = false;
    int64_t mat = 0, bnd = 0, ops = 0, segops = 0, segctl = 0;
    while (end < dp.size()) {
      const PairWork& w = dp[end];
      const int64_t need = (mat + w.mat_dw) * 4 + (bnd + w.bnd_gr) * 8 + 3 * (ops + w.ops_b) + segops + w.segops_b +
                           segctl + w.segctl_b + 8192;
      if ((need > c->budget || lin_all) && end > pos) break;
      if (need > c->budget || lin_all) {  // a pair whose matrix does not fit: linear-space traceback (f2)
        if (c->opts.linear_space < 0 || sc.affine)
          return fail(NWK_ENOMEM, "pair %lld (%d x %d) needs %lld bytes > HBM budget %lld", (long long)w.id,
                      w.m, w.n, (long long)need, (long long)c->budget);
        lin_one = true;
        break;
      }
      mat += w.mat_dw; bnd += w.bnd_gr; ops += w.ops_b; segops += w.segops_b; segctl += w.segctl_b;
      ++end;
    }
    if (lin_one) {
      fin.join();
      // forced (tests): as many pairs per linear-space batch as fit; automatic:
      // the pair that does not fit, alone, with as many bands per group as fit
      const Plan lpl = lin_plan(pl);
      const int G = lin_all ? c->opts.linear_space : lin_auto_groups(c, lpl, dp[pos]);
      if (G < 1)
        return fail(NWK_ENOMEM, "pair (%d x %d): boundary rows and two bands exceed the HBM budget %lld", dp[pos].m,
                    dp[pos].n, (long long)c->budget);
      size_t lend = pos + 1;
      int64_t used = lin_geo(lpl, dp[pos], G).bytes;
      while (lin_all && lend < dp.size()) {
        const int64_t more = lin_geo(lpl, dp[lend], G).bytes;
        if (used + more + 8192 > c->budget) break;
        used += more;
        ++lend;
      }
      const int nl = (int)(lend - pos);
      std::vector<Finalized> fs((size_t)nl);
      if ((rc = align_linear_batch(c, pl, sc, dp.data() + pos, nl, G, fs.data(), a1, a2, &st)) != NWK_OK) return rc;
      for (int q = 0; q < nl; ++q) {
        const PairWork& w = dp[pos + q];
        penalties[w.out] = fs[q].penalty;
        memcpy(hashes + 64 * w.out, fs[q].hash, 64);
        if (chain) chain->ready[w.out] = 1;
        mark_ready(c, w.out);
      }
      if (chain) chain->advance();
      pos = lend;
      continue;
    }
    const int np = (int)(end - pos);
    const double tb0 = now_ms();
    bool devhash = false;
    if (dev_ok) {
      double bytes = 0, maxlen = 0;
      for (size_t q = pos; q < end; ++q) {
        bytes += 2.0 * (dp[q].m + dp[q].n);
        maxlen = std::max(maxlen, (double)(dp[q].m + dp[q].n));
      }
      const double waves = 2.0 * np / 64.0, slots = 8.0 * c->cus;
      // ~0.007 ms per 128-byte block of the longest row since nw_rows / nw_hash
      // went to four waves per pair and bitop3 rounds (C3: 781 blocks, 5.5 ms)
      const double est_dev = (maxlen / 128.0) * 0.007 * std::max(1.0, waves / slots);
      const double est_host = bytes / (350e3 * c->host_threads);
      devhash = fin_mode == 1 || est_dev < 0.8 * est_host;
      // nw_align_col under "auto": the device finalize runs after the launch (a
      // row's SHA-512 is one lane's serial chain: ~4.4 ms for C3's 100 KB rows),
      // while the streamed host finalize (hstream below) takes each pair as its
      // walk ends, during the launch -- only the last pair's ~0.3 ms is left
      // after it.  So host threads finalize wherever they keep up with the fill
      // (estimated: cells at ~30 TCUPS, or the longest pair's span at ~0.27 us
      // per step): C3's 8-rank shard 35 -> ~31 ms; C4 (1 GB of rows) stays on
      // the device.
      static const int hstream_auto = getenv("NWK_HOST_STREAM") ? atoi(getenv("NWK_HOST_STREAM")) : 1;
      if (devhash && fin_mode < 0 && pl.mode == kCol && hstream_auto != 0) {
        double cells = 0, span = 0;
        for (size_t q = pos; q < end; ++q) {
          cells += (double)dp[q].m * dp[q].n;
          span = std::max(span, (double)dp[q].n + 100.0 * (double)ceil_div(dp[q].m, kBitsRows));
        }
        const double est_fill = std::max(cells / 3.0e10, span * 0.27e-3);
        if (est_host < 0.5 * est_fill) devhash = false;
      }
      st.device_finalized += devhash ? 1 : 0;
    }
    // Layout: [granules | slack | matrices | op strings].  The granule region
    // always starts at offset 0, so across batches it only ever overlaps
    // older granules or zeros -- never stale matrix words, whose upper halves
    // could equal a future epoch tag.  Bytes past the previous batch's
    // granule region are zeroed before they are used as granules.
    const int64_t bnd_need_b = bnd * 8 + 4096;  // + slack: band 0's dummy prefetches
    const int64_t mat_base_b = round_up(bnd_need_b, 256);
    const int64_t ops_base_b = round_up(mat_base_b + mat * 4, 256);
    const int64_t segops_base_b = round_up(ops_base_b + ops, 256);
    // device finalize rows (align1 | align2, op-region layout) + 256 B read slack each
    const int64_t rows_base_b = round_up(segops_base_b + segops, 256);
    const int64_t work_b = rows_base_b + 2 * (ops + 256) + 256;  // + slack: traceback tile overrun of the last band
    void* const old_work = c->d_work.p;
    if ((rc = c->d_work.ensure((size_t)work_b)) != NWK_OK) return rc;
    if (c->d_work.p != old_work) c->clean_b = 0;
    if (bnd_need_b > c->clean_b) {
      HIP_TRY(hipMemsetAsync(c->d_work.as<uint8_t>() + c->clean_b, 0, (size_t)(bnd_need_b - c->clean_b), c->stream));
    }
    c->clean_b = bnd_need_b;
    // debug: NWK_POISON_BATCH=<byte> fills this batch's matrix region before the
    // launch, so a walk reading a cell no band of this batch wrote reads that byte
    // (for nw_align_pka 0x22 is tag 2, a code the fill never writes: the walk fails)
    static const int poison_batch = getenv("NWK_POISON_BATCH") ? atoi(getenv("NWK_POISON_BATCH")) : -1;
    if (poison_batch >= 0 && mat > 0)
      HIP_TRY(hipMemsetAsync(c->d_work.as<uint8_t>() + mat_base_b, poison_batch & 0xff, (size_t)mat * 4, c->stream));
    // ---- descriptors and dependency-ordered band tasks (band-major)
    const int par = st.batches & 1;  // host buffer set of this batch
    if ((rc = c->h_pairs[par].ensure(sizeof(PairDesc) * np)) != NWK_OK) return rc;
    PairDesc* pd = c->h_pairs[par].as<PairDesc>();
    int64_t mo = 0, bo = 0, oo = 0, ntasks = 0, so = 0, ro = 0, nsegs = 0, njobs = 0;
    int maxb = 0;
    for (int q = 0; q < np; ++q) {
      const PairWork& w = dp[pos + q];
      PairDesc& d = pd[q];
      d.x_off = c->c_off[w.i];
      d.y_off = c->c_off[w.j];
      d.e_off = bitsy || gotoh ? c->yw_off[w.j] : c->e_off[w.j];
      d.xw_off = pl.mode == kBitsStrip ? c->yw_off[w.i] : 0;
      d.bits_np = pl.mode == kBitsStrip ? strip_np(w.n) : 0;
      d.prio = 0;
      d.mat_off = mat_base_b / 4 + mo;
      d.bnd_off = bo;
      d.ops_off = ops_base_b + oo;
      d.m = w.m;
      d.n = w.n;
      d.nbands = (int)ceil_div(w.m, bitsy || gotoh ? kBitsRows : kBandRows);
      d.nchunks = pl.mode == kBitsStrip ? d.bits_np / 64 : gotoh ? (w.n >> 5) + 1 : (int)ceil_div(w.n, 64);
      d.sblocks = pl.mode == kBits        ? bits_sblocks(d.nchunks)
                  : pl.mode == kCol       ? col_sblocks(d.nchunks)
                  : pl.mode == kBitsStrip ? strip_sblocks(w.m, w.n)
                                          : sblocks_of(pl.mode, d.nchunks);
      d.bits_w = w.bits_w;
      d.bits_nblk = w.bits_nblk;
      d.slot = q;
      d.spec_every = w.spec;
      d.nguess = w.nguess;
      d.task_off = ntasks;  // one tdone entry per task
      d.seg_off = nsegs;    // nguess seginfo entries per task (kCol: one per band but the last)
      d.rec_off = ro;
      d.segops_off = so;
      if (pl.mode == kCol) {
        const int64_t nseg = w.spec > 0 ? d.nbands - 1 : 0;
        nsegs += nseg;
        ro += nseg * kBitsRows;  // a record per row of each segment's band
      } else {
        nsegs += tasks_of(pl.mode, d.nbands) * w.nguess;
        ro += 32 * (w.m / 128 + 1);
      }
      njobs += w.njobs;
      so += w.segops_b;
      mo += w.mat_dw; bo += w.bnd_gr; oo += w.ops_b;
      ntasks += tasks_of(pl.mode, d.nbands);
      maxb = std::max(maxb, (int)tasks_of(pl.mode, d.nbands));
    }
    // kCol, span-bound batches (under two rounds of tasks per wave slot, e.g.
    // big13): a pair costs at least its span n + ~100 x bands steps, so the
    // pairs with the longest spans get issue priority over the rest (their
    // waves then step at nearly a lone wave's rate).  NWK_COL_PRIO=0 disables.
    static const int col_prio_env = getenv("NWK_COL_PRIO") ? atoi(getenv("NWK_COL_PRIO")) : 1;
    if (pl.mode == kCol && col_prio_env != 0 && ntasks <= 2 * (int64_t)grid * 4) {
      double smax = 0;
      for (int q = 0; q < np; ++q) smax = std::max(smax, (double)pd[q].n + 100.0 * pd[q].nbands);
      for (int q = 0; q < np; ++q) pd[q].prio = (double)pd[q].n + 100.0 * pd[q].nbands >= 0.7 * smax ? 2 : 0;
    }
    // kCol streamed batches (fused finalize: records leave during the launch;
    // a sharded rank's pairs come in canonical order): the first 1/8 of the
    // pairs dequeued fill at issue priority 2 and the next 1/8 at 1, so the
    // lowest canonical ids are out early and rank 0's chain (which consumes
    // them one record at a time, dist.align_sharded_records) starts on them
    // while the rest fills.  NWK_PIECE_PRIO=0 disables.
    static const int piece_prio_env = getenv("NWK_PIECE_PRIO") ? atoi(getenv("NWK_PIECE_PRIO")) : 1;
    // (want_fuse: the fused finalize below, asked for or automatic)
    static const int auto_fuse_env = getenv("NWK_AUTO_FUSE") ? atoi(getenv("NWK_AUTO_FUSE")) : 1;
    const bool want_fuse = devhash && bitsy && !sc.affine &&
                           (c->opts.finalize == 3 ||
                            (c->opts.finalize == 0 && auto_fuse_env != 0 && chain && pl.mode == kCol && np >= 8192));
    // (the first np / div pairs at priority 2, the next np / div at 1; NWK_PIECE_DIV, default 8:
    // C4 at 8 ranks, chain end 19.85 ms with div 16, 19.05 with 8, 19.63 with 6, profiles/r06/c4_records.txt)
    // NWK_PIECE_TOP (experiment, default 2): the first tier's priority; each next
    // np / div pairs one lower, down to 1 (3: the first tier issues level with the walks)
    static const int piece_div_env = getenv("NWK_PIECE_DIV") ? std::max(2, atoi(getenv("NWK_PIECE_DIV"))) : 8;
    static const int piece_top_env = getenv("NWK_PIECE_TOP") ? std::min(3, std::max(1, atoi(getenv("NWK_PIECE_TOP")))) : 2;
    if (pl.mode == kCol && piece_prio_env != 0 && want_fuse && c->opts.finalize == 3 && np >= 32) {
      const int tier = std::max(1, np / piece_div_env);
      for (int q = 0; q < np; ++q) {
        const int pr = piece_top_env - q / tier;
        if (pr >= 1) pd[q].prio = std::max(pd[q].prio, pr);
      }
    }
    if ((rc = c->h_tasks.ensure(sizeof(int2) * ntasks)) != NWK_OK) return rc;
    int2* tk = c->h_tasks.as<int2>();
    // Pair-major (pairs already largest first): a pair's bands are dequeued
    // together, so pairs finish one after another and each one's traceback
    // runs concurrently with the fill of the pairs after it.
    // nw_align_bits with more than one round of tasks per wave slot: band-major.
    // Its bands trail each other by 2048 + 64 steps, so bands of one pair
    // dequeued together wait b x 2112 steps; band-major spaces them by a round
    // of other pairs' bands (C3: 11.5k -> 14.0k GCUPS; C3's 8-rank shard, 1.5
    // rounds: 59 -> 51 ms; big13, under one round: pair-major 40 vs 44 ms).
    // NWK_ORDER overrides (0 pair-major, 1 band-major, g >= 2 groups of g
    // pairs, band-major inside).
    int64_t t = 0;
    static const int order_env = getenv("NWK_ORDER") ? atoi(getenv("NWK_ORDER")) : -1;
    int order = order_env;
    if (order < 0 && pl.mode == kBits && c->opts.task_order > 0) order = c->opts.task_order == 1 ? 0 : 1;
    if (order < 0) order = (pl.mode == kBits || pl.mode == kAffinePk || gotoh) && ntasks > 4 * (int64_t)grid ? 1 : 0;
    if (pl.mode == kBitsStrip) order = 0;  // one task per pair, largest first
    // kCol: bands trail each other by ~96 steps, so a pair's bands dequeued
    // together run as one short pipeline: pair-major unless NWK_ORDER says otherwise
    if (pl.mode == kCol && order_env < 0) order = c->opts.task_order == 2 ? 1 : 0;
    if (order == 1) {  // band-major (experiment)
      for (int b = 0; b < maxb; ++b)
        for (int q = 0; q < np; ++q)
          if (b < tasks_of(pl.mode, pd[q].nbands)) tk[t++] = make_int2(q, b);
    } else if (order >= 2) {  // groups of `order` pairs, band-major inside a group (experiment)
      for (int g0 = 0; g0 < np; g0 += order) {
        const int g1 = std::min(np, g0 + order);
        int mb = 0;
        for (int q = g0; q < g1; ++q) mb = std::max(mb, (int)tasks_of(pl.mode, pd[q].nbands));
        for (int b = 0; b < mb; ++b)
          for (int q = g0; q < g1; ++q)
            if (b < tasks_of(pl.mode, pd[q].nbands)) tk[t++] = make_int2(q, b);
      }
    } else {
      for (int q = 0; q < np; ++q)
        for (int b = 0; b < tasks_of(pl.mode, pd[q].nbands); ++b) tk[t++] = make_int2(q, b);
    }
    if ((rc = c->d_pairs.ensure(sizeof(PairDesc) * np)) != NWK_OK) return rc;
    if ((rc = c->d_tasks.ensure(sizeof(int2) * ntasks)) != NWK_OK) return rc;
    if ((rc = c->d_oplen.ensure(sizeof(int) * np)) != NWK_OK) return rc;
    if ((rc = c->d_endij.ensure(sizeof(int2) * np)) != NWK_OK) return rc;
    if ((rc = c->d_done.ensure(sizeof(unsigned) * np)) != NWK_OK) return rc;
    if ((rc = c->d_retry.ensure(sizeof(int) * np)) != NWK_OK) return rc;
    if ((rc = c->h_retry.ensure(sizeof(int) * np)) != NWK_OK) return rc;
    if ((rc = c->h_oplen[par].ensure(sizeof(int) * np)) != NWK_OK) return rc;
    if ((rc = c->h_endij[par].ensure(sizeof(int2) * np)) != NWK_OK) return rc;
    if ((rc = c->h_ops[par].ensure((size_t)ops)) != NWK_OK) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_pairs.p, pd, sizeof(PairDesc) * np, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->d_tasks.p, tk, sizeof(int2) * ntasks, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_ctl.p, 0, 256, c->stream));
    HIP_TRY(hipMemsetAsync(c->d_done.p, 0, sizeof(unsigned) * np, c->stream));
    bool windowed = false;
    for (int q = 0; q < np && !windowed; ++q) windowed = pd[q].bits_w > 0;
    // fill-vs-walk guard (skel:274): the kernels that give their H(m, n) per
    // pair (FillArgs::endv); NWK_GUARD=0 disables (A/B)
    const bool guard = guard_on && guard_mode(pl.mode) && !(getenv("NWK_AFF_NOTRACE") || getenv("NWK_NOTRACE"));
    if (guard) {
      st.guard_checked += np;
      if ((rc = c->d_endv.ensure(sizeof(int) * np)) != NWK_OK) return rc;
      if ((rc = c->h_endv[par].ensure(sizeof(int) * np)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_endv.p, 0, sizeof(int) * np, c->stream));
    }
    if (windowed || guard) HIP_TRY(hipMemsetAsync(c->d_retry.p, 0, sizeof(int) * np, c->stream));
    // [tdone u32 | seginfo 8 x int | recs u64 | job ready u32 | head, tail | jobs int2]
    const int64_t seginfo_base_b = ntasks * 4;
    const int64_t rec_base_b = round_up(seginfo_base_b + nsegs * 32, 8);
    const int64_t tjr_base_b = rec_base_b + ro * 8;
    const int64_t tjc_base_b = tjr_base_b + njobs * 4;
    const int64_t tj_base_b = round_up(tjc_base_b + 8, 8);
    const int64_t segctl_b = tj_base_b + njobs * 8;
    if (segmented(pl.mode)) {
      if ((rc = c->d_segctl.ensure((size_t)segctl_b)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_segctl.p, 0, (size_t)segctl_b, c->stream));
      c->colseg_clean_b = 0;
    }
    // kCol segments: records (u64) in d_segctl, info (int4) in d_colinfo.  A
    // record counts only with this launch's epoch tag (20 bits), so the record
    // buffer is cleared only where it may hold anything else: fresh or grown
    // memory, another mode's data, or once every 2^20 launches (the tag wraps).
    // The info is cleared per batch (its flag is a whole epoch).
    const bool colseg = pl.mode == kCol && nsegs > 0;
    const int64_t colseg_ctl_b = ro * 8;
    if (colseg) {
      if ((rc = c->d_colinfo.ensure((size_t)nsegs * 16)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_colinfo.p, 0, (size_t)nsegs * 16, c->stream));
      void* const old_ctl = c->d_segctl.p;
      if ((rc = c->d_segctl.ensure((size_t)colseg_ctl_b)) != NWK_OK) return rc;
      if (c->d_segctl.p != old_ctl || c->epoch + 2u - c->colseg_epoch0 >= (1u << 20)) c->colseg_clean_b = 0;
      if (c->colseg_clean_b == 0) c->colseg_epoch0 = c->epoch;
      if (colseg_ctl_b > c->colseg_clean_b) {
        HIP_TRY(hipMemsetAsync(c->d_segctl.as<uint8_t>() + c->colseg_clean_b, 0, (size_t)(colseg_ctl_b - c->colseg_clean_b),
                               c->stream));
        c->colseg_clean_b = colseg_ctl_b;
      }
    }

    FillArgs fa{};
    fa.pairs = c->d_pairs.as<PairDesc>();
    fa.tasks = c->d_tasks.as<int2>();
    fa.ntasks = (int)ntasks;
    fa.codes = c->d_codes[pl.kind].as<uint8_t>();
    fa.E = c->d_E[pl.kind].as<uint32_t>();
    fa.sel = pl.mode == kPacked    ? c->d_sel[pl.K0 < 0 ? 1 : 0].as<uint32_t>()
             : band_pairs(pl.mode) ? c->d_sel[2 + (pl.K0 < 0 ? 1 : 0)].as<uint32_t>()
                                   : nullptr;
    fa.mat = c->d_work.as<uint32_t>();
    fa.bnd = c->d_work.as<unsigned long long>();
    fa.counter = c->d_ctl.as<unsigned>();
    fa.err = c->d_ctl.as<unsigned>() + 16;
    fa.done = c->d_done.as<unsigned>();
    fa.epoch = ++c->epoch;
    if (fa.epoch == 0) fa.epoch = ++c->epoch;
    fa.K0 = pl.K0;
    fa.K1 = pl.K1;
    fa.go = sc.go;
    fa.dbg_notrace = (getenv("NWK_AFF_NOTRACE") || getenv("NWK_NOTRACE")) ? 1 : 0;
    fa.dbg_badwalk = getenv("NWK_DBG_BADWALK") ? atoi(getenv("NWK_DBG_BADWALK")) : 0;
    static const int band_prio_env = getenv("NWK_BAND_PRIO") ? atoi(getenv("NWK_BAND_PRIO")) : 0;
    fa.band_prio = band_prio_env;
    fa.lin_mode = 0;
    fa.prog = nullptr;
    fa.yw = bitsy || gotoh ? c->d_yw.as<unsigned>() : nullptr;
    fa.strip_ring = strip_ring;
    fa.retry = c->d_retry.as<int>();
    fa.endv = guard ? c->d_endv.as<int>() : nullptr;
    fa.pxy = sc.pxy;
    fa.pgap = sc.pgap;
    // (tests) NWK_DBG_CORRUPT = slot + 1: the first batch of the call (every batch with
    // NWK_DBG_CORRUPT_ALL) flips the stored code of cell (m, n) of that pair before its walk
    fa.dbg_corrupt = (st.batches == 0 || getenv("NWK_DBG_CORRUPT_ALL")) && getenv("NWK_DBG_CORRUPT")
                         ? atoi(getenv("NWK_DBG_CORRUPT")) : 0;
    // streamed shards (finalize "fused" asked for): the first two pieces' pairs
    // (prio >= 1 above) are hashed by their tracing wave at once, not in groups
    // of 32 (the chain on rank 0 waits for the lowest canonical ids).
    // NWK_EARLY_HASH=0 off, p > 0: prio >= p.
    static const int early_env = getenv("NWK_EARLY_HASH") ? atoi(getenv("NWK_EARLY_HASH")) : 1;
    fa.early_hash = c->opts.finalize == 3 ? early_env : 0;
    if (getenv("NWK_WATCHDOG")) {
      if ((rc = c->d_prog.ensure(4 * (size_t)(grid + 1) * 4)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_prog.p, 0, 4 * (size_t)(grid + 1) * 4, c->stream));
      fa.prog = c->d_prog.as<unsigned>();
    }
    fa.ge = sc.ge;
    fa.stamps = nullptr;
    fa.ntasks_pairs = np;
    if (c->opts.verbose >= 2) {
      if ((rc = c->d_stamps.ensure(88 * (size_t)np + 16 + 16 * (size_t)np)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_stamps.as<uint8_t>() + 88 * (size_t)np + 8, 0, 16 * (size_t)np, c->stream));
      HIP_TRY(hipMemsetAsync(c->d_stamps.p, 0, 88 * (size_t)np, c->stream));
      HIP_TRY(hipMemsetAsync(c->d_stamps.as<uint8_t>() + 88 * (size_t)np, 0xff, 8, c->stream));  // kernel start: atomicMin
      fa.stamps = c->d_stamps.as<unsigned long long>();
    }
    fa.ops = c->d_work.as<uint8_t>();
    const bool seg = segmented(pl.mode);
    fa.tdone = seg ? c->d_segctl.as<unsigned>() : nullptr;
    fa.seginfo = seg ? reinterpret_cast<int*>(c->d_segctl.as<uint8_t>() + seginfo_base_b) : nullptr;
    fa.recs = seg ? reinterpret_cast<unsigned long long*>(c->d_segctl.as<uint8_t>() + rec_base_b) : nullptr;
    if (colseg) {
      fa.recs = c->d_segctl.as<unsigned long long>();
      fa.seginfo = c->d_colinfo.as<int>();
    }
    fa.tj_ready = seg ? reinterpret_cast<unsigned*>(c->d_segctl.as<uint8_t>() + tjr_base_b) : nullptr;
    fa.tj_head = seg ? reinterpret_cast<unsigned*>(c->d_segctl.as<uint8_t>() + tjc_base_b) : nullptr;
    fa.tj_tail = seg ? fa.tj_head + 1 : nullptr;
    fa.tjobs = seg ? reinterpret_cast<int2*>(c->d_segctl.as<uint8_t>() + tj_base_b) : nullptr;
    fa.ntjobs = seg ? (int)njobs : 0;
    fa.segops = c->d_work.as<uint8_t>() + segops_base_b;
    fa.oplen = c->d_oplen.as<int>();
    fa.endij = c->d_endij.as<int2>();
    // finalize 3: the bits kernels' device finalize fused into the fill launch
    // (rows by the tracing wave, SHA-512 by waves that claim 32 traced pairs
    // from a queue: nwk_bits.hip fin_rows / hq_hash), records streaming to the
    // host while it runs.  On request (a rank of a sharded job exchanges and
    // chains finished pairs early); not for nw_align_bits on one GPU, where the
    // separate nw_rows + nw_hash is faster (C3 161.5 vs 165.4 ms per step).
    // Automatic for nw_align_col getMinimumPenalties-style calls of >= 8,192
    // pairs in a batch (C4: 32,640): with the separate finalize the chain's
    // ~12.5 ms ran after the launch; with records streaming out of it the host
    // chains while the launch runs.  NWK_AUTO_FUSE=0 disables.
    const bool fuse = want_fuse && !fa.dbg_notrace;
    if (devhash) {
      if ((rc = c->d_pen.ensure(4 * (size_t)np)) != NWK_OK) return rc;
      if ((rc = c->d_hash.ensure(64 * (size_t)np)) != NWK_OK) return rc;
    }
    unsigned* rflag = nullptr;
    int* rpen = nullptr;
    uint8_t* rhash = nullptr;
    if (fuse) {
      const size_t rb = (size_t)np * 72;
      if ((rc = c->h_rec[par].ensure(rb, hipHostMallocMapped | hipHostMallocCoherent)) != NWK_OK) return rc;
      rflag = c->h_rec[par].as<unsigned>();
      rpen = reinterpret_cast<int*>(rflag + np);
      rhash = reinterpret_cast<uint8_t*>(rpen + np);
    }
    if (fuse) {
      fa.fuse_fin = 1;
      fa.pxy = sc.pxy;
      fa.pgap = sc.pgap;
      fa.raw = c->d_codes[1].as<uint8_t>();
      fa.ops_base = ops_base_b;
      fa.rows1 = c->d_work.as<uint8_t>() + rows_base_b;
      fa.rows2 = fa.rows1 + ops + 256;
      void *dflag = nullptr;
      HIP_TRY(hipHostGetDevicePointer(&dflag, rflag, 0));
      fa.fin_flag = static_cast<unsigned*>(dflag);
      fa.fin_pen = reinterpret_cast<int*>(fa.fin_flag + np);
      fa.fin_hash = reinterpret_cast<uint8_t*>(fa.fin_pen + np);
      if ((rc = c->d_hq.ensure((8 + 8) * (size_t)np)) != NWK_OK) return rc;  // queue | row lengths, penalties
      fa.hq = c->d_hq.as<unsigned long long>();
      fa.fin_len = reinterpret_cast<int*>(fa.hq + np);
      fa.hq_ctl = c->d_ctl.as<unsigned>() + 32;  // (d_ctl's 256 bytes are zeroed per batch)
    }
    // Streamed host finalize (nw_align_col batches finalized on the host: few
    // long pairs, big13): the pair walk writes its moves into host-mapped
    // memory and flags the pair, and host threads build rows and hashes while
    // the launch still runs -- the pairs traced first (big13: 8 ms into a
    // 24 ms launch) are done before it ends.  NWK_HOST_STREAM=0 disables.
    static const int hstream_env = getenv("NWK_HOST_STREAM") ? atoi(getenv("NWK_HOST_STREAM")) : 1;
    const bool hstream = pl.mode == kCol && !devhash && !fuse && a1 == nullptr && hstream_env != 0 && !fa.dbg_notrace;
    fa.ops_host = nullptr;
    fa.host_rec = nullptr;
    if (hstream) {
      if ((rc = c->h_opsm[par].ensure((size_t)ops + 256, hipHostMallocMapped | hipHostMallocCoherent)) != NWK_OK) return rc;
      const size_t hrb = sizeof(int) * kHostRecInts * (size_t)np;
      if ((rc = c->h_hrec[par].ensure(hrb, hipHostMallocMapped | hipHostMallocCoherent)) != NWK_OK) return rc;
      memset(c->h_hrec[par].p, 0, hrb);
      void *dops = nullptr, *drec = nullptr;
      HIP_TRY(hipHostGetDevicePointer(&dops, c->h_opsm[par].p, 0));
      HIP_TRY(hipHostGetDevicePointer(&drec, c->h_hrec[par].p, 0));
      fa.ops_host = static_cast<uint8_t*>(dops);
      fa.host_rec = static_cast<int*>(drec);
      fa.ops_base = ops_base_b;
    }
    // One persistent launch: fill bands, and each pair's traceback runs on
    // the wave that finishes the pair's last band (nw_align).
    if (c->opts.verbose >= 3) {
      fprintf(stderr, "nwk batch %d: pairs [%zu, %zu) ids %lld..%lld, %lld tasks, work %.3f GB (mat %.3f, bnd %.3f, ops %.3f)\n",
              st.batches, pos, end, (long long)dp[pos].id, (long long)dp[end - 1].id, (long long)ntasks, work_b / 1e9,
              mat * 4 / 1e9, bnd * 8 / 1e9, ops / 1e9);
      fflush(stderr);
    }
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    if (pl.mode == kBits)
      HIP_TRY(launch_bits(fa, sc.pxy, sc.pgap, (int)std::min<int64_t>(grid, ceil_div(ntasks, 4)), c->stream));
    else if (pl.mode == kCol) {
      // the plain (not fused) instantiation at 5 waves/SIMD (nwk_col.hip
      // NWK_COL_WPE_HI): C3's 4-rank shard 60.5 -> 48.6 ms; NWK_COL_WPE_HI=0: 4
      static const int wpe_hi_env = getenv("NWK_COL_WPE_HI") ? atoi(getenv("NWK_COL_WPE_HI")) : 1;
      const bool hi = !fuse && wpe_hi_env != 0;
      const int gcol = col_blocks_per_cu(sc.pgap, hi) * c->cus;
      HIP_TRY(launch_col(fa, sc.pxy, sc.pgap, (int)std::min<int64_t>(gcol, ceil_div(ntasks, 4)), hi, c->stream));
    }
    else if (pl.mode == kBitsStrip)
      HIP_TRY(launch_strip(fa, sc.pxy, sc.pgap, (int)std::min<int64_t>(grid, ceil_div(ntasks, 4)), c->stream));
    else if (gotoh)
      HIP_TRY(launch_gotoh(fa, sc.pxy, sc.go, sc.ge, (int)std::min<int64_t>(grid, ceil_div(ntasks, 4)), c->stream));
    else
      HIP_TRY(launch_fill(pl.mode, pl.bits, fa, std::min<int64_t>(grid, ceil_div(ntasks, 4)), c->stream));
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    if (seg) HIP_TRY(launch_gather(fa, np, pl.mode == kPacked2 ? 1 : 0, c->stream));  // segment chains -> op strings
    if (devhash && !fuse) {
      HashArgs ha;
      ha.pairs = fa.pairs;
      ha.npairs = np;
      ha.raw = c->d_codes[1].as<uint8_t>();
      ha.ops = fa.ops;
      ha.ops_base = ops_base_b;
      ha.rows1 = c->d_work.as<uint8_t>() + rows_base_b;
      ha.rows2 = ha.rows1 + ops + 256;
      ha.oplen = fa.oplen;
      ha.endij = fa.endij;
      ha.pxy = sc.pxy;
      ha.gopen = sc.affine ? sc.go + sc.ge : sc.pgap;
      ha.gext = sc.affine ? sc.ge : sc.pgap;
      ha.penalties = c->d_pen.as<int>();
      ha.hashes = c->d_hash.as<uint8_t>();
      ha.endv = fa.endv;
      ha.retry = fa.retry;
      HIP_TRY(launch_hash(ha, c->stream));
    }
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    // Fused finalize: a host thread takes each pair's record as its flag
    // arrives (host-mapped, written by the wave that traced the pair) and
    // feeds the chain while the launch still runs.
    std::shared_ptr<FusedSync> fsync;
    struct FuseGuard {  // an early return abandons the consumer instead of leaving it waiting
      std::shared_ptr<FusedSync>* f;
      ~FuseGuard() {
        int z = 0;
        if (*f) (*f)->done.compare_exchange_strong(z, 2);
      }
    } fguard{&fsync};
    if (fuse) {
      fin.join();
      fsync = std::make_shared<FusedSync>();
      const PairWork* dwf = dp.data() + pos;  // (dp never reallocates: reserved for every re-run)
      const unsigned ep = fa.epoch;
      fin.start([c, np, dwf, fsync, ep, rflag, rpen, rhash, penalties, hashes, chain]() {
        std::vector<char> got((size_t)np, 0);
        int64_t lo = 0, ngot = 0;
        for (;;) {
          const int d = fsync->done.load(std::memory_order_acquire);
          if (d == 2) return;
          bool any = false;
          const int64_t hi = d ? np : std::min<int64_t>(np, lo + 8192);
          for (int64_t q = lo; q < hi; ++q) {
            if (got[(size_t)q] || __atomic_load_n(rflag + q, __ATOMIC_ACQUIRE) != ep) continue;
            const PairWork& w = dwf[q];
            penalties[w.out] = rpen[q];
            memcpy(hashes + 64 * w.out, rhash + 64 * q, 64);
            if (chain) {
              chain->prepare(w.out);
              chain->ready[w.out] = 1;
            }
            mark_ready(c, w.out);
            got[(size_t)q] = 1;
            ++ngot;
            any = true;
          }
          while (lo < np && got[(size_t)lo]) ++lo;
          if (chain && any) chain->advance();
          if (d || ngot == np) break;
          if (!any) std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
        // every pair without a record must be a window re-run
        if (ngot < np) {
          while (fsync->done.load(std::memory_order_acquire) == 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
          if (fsync->done.load() == 2) return;
          for (int64_t q = 0; q < np; ++q)
            if (!got[(size_t)q] && !(!fsync->skip.empty() && fsync->skip[(size_t)q])) ++fsync->missing;
        }
      });
    }
    if (hstream) {
      fin.join();
      fsync = std::make_shared<FusedSync>();
      const PairWork* dwf = dp.data() + pos;
      const PairDesc* pdh = pd;  // (h_pairs[par] stays until batch b + 2)
      const unsigned ep = fa.epoch;
      const int* hrec = c->h_hrec[par].as<int>();
      const uint8_t* hops = c->h_opsm[par].as<uint8_t>();
      const int64_t obase = ops_base_b;
      GuardLog* glog = &gl;
      const bool gchk = guard;
      const int64_t gpos = (int64_t)pos;
      fin.start([c, np, dwf, pdh, fsync, ep, hrec, hops, obase, sc, penalties, hashes, chain, glog, gchk, gpos]() {
        // state per pair: 0 pending, 1 claimed, 2 finalized, 3 left the window (re-run), 4 the
        // walk failed (length -2: the launch reports the error; the pair is never finalized,
        // reported or chained), 5 its path's cost is not the fill's H(m, n) (guard: re-run)
        std::unique_ptr<std::atomic<int>[]> state(new std::atomic<int>[(size_t)np]);
        for (int64_t q = 0; q < np; ++q) state[q].store(0, std::memory_order_relaxed);
        std::atomic<int64_t> nleft{np};
        auto work = [&]() {
          for (;;) {
            const int d = fsync->done.load(std::memory_order_acquire);
            if (d == 2 || nleft.load(std::memory_order_acquire) == 0) return;
            bool any = false;
            for (int64_t q = 0; q < np; ++q) {
              const int* hr = hrec + kHostRecInts * q;
              if (state[q].load(std::memory_order_relaxed) != 0 || __atomic_load_n(hr, __ATOMIC_ACQUIRE) != (int)ep)
                continue;
              int z = 0;
              if (!state[q].compare_exchange_strong(z, 1)) continue;
              any = true;
              const int len = hr[1];
              if (len < 0) {
                state[q].store(len == -1 ? 3 : 4, std::memory_order_release);
              } else {
                const PairWork& w = dwf[q];
                Finalized f;
                finalize_pair(c->seqs.data() + c->off[w.i], w.m, c->seqs.data() + c->off[w.j], w.n, sc,
                              hops + (pdh[q].ops_off - obase), len, hr[2], hr[3], &f);
                if (gchk && f.penalty != hr[4]) {
                  glog->add(gpos + q, hr[4], f.penalty);
                  state[q].store(5, std::memory_order_release);
                } else {
                  penalties[w.out] = f.penalty;
                  memcpy(hashes + 64 * w.out, f.hash, 64);
                  state[q].store(2, std::memory_order_release);
                }
              }
              nleft.fetch_sub(1, std::memory_order_acq_rel);
            }
            if (!any) {
              if (d == 1) return;  // the launch is over: every flag that will come has come
              std::this_thread::sleep_for(std::chrono::microseconds(20));
            }
          }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < c->host_threads; ++t) pool.emplace_back(work);
        // this thread: finalizes too, and reports finished pairs in slot order to the chain
        std::vector<char> told((size_t)np, 0);
        int64_t lo = 0;
        auto report = [&]() {
          bool any = false;
          for (int64_t q = lo; q < np; ++q) {
            if (told[(size_t)q] || state[q].load(std::memory_order_acquire) != 2) continue;
            const PairWork& w = dwf[q];
            if (chain) {
              chain->prepare(w.out);
              chain->ready[w.out] = 1;
            }
            mark_ready(c, w.out);
            told[(size_t)q] = 1;
            any = true;
          }
          while (lo < np && (told[(size_t)lo] || state[lo].load(std::memory_order_acquire) == 3 ||
                             state[lo].load(std::memory_order_acquire) == 5))
            ++lo;
          if (chain && any) chain->advance();
        };
        std::thread rep_thread;
        std::atomic<int> stop{0};
        rep_thread = std::thread([&]() {
          while (!stop.load(std::memory_order_acquire)) {
            report();
            std::this_thread::sleep_for(std::chrono::microseconds(50));
          }
          report();
        });
        work();
        for (auto& t : pool) t.join();
        stop.store(1, std::memory_order_release);
        rep_thread.join();
        if (fsync->done.load() == 2) return;
        while (fsync->done.load(std::memory_order_acquire) == 0) std::this_thread::sleep_for(std::chrono::microseconds(20));
        if (fsync->done.load() == 2) return;
        for (int64_t q = 0; q < np; ++q) {
          const int st_q = state[q].load();
          const bool skipped = !fsync->skip.empty() && fsync->skip[(size_t)q];
          if ((st_q != 2 && st_q != 5 && !skipped) || (st_q == 2 && skipped)) ++fsync->missing;
        }
      });
    }
    if (c->opts.verbose >= 3) {
      fprintf(stderr, "nwk batch %d: launched mode %d bits %d grid %d, waiting\n", st.batches, pl.mode, pl.bits, grid);
      fflush(stderr);
    }
    static const int watchdog = getenv("NWK_WATCHDOG") ? atoi(getenv("NWK_WATCHDOG")) : 0;
    if (watchdog > 0) {  // debug: report where a launch that does not finish is stuck, then exit
      const double t0 = now_ms();
      while (hipStreamQuery(c->stream) == hipErrorNotReady && now_ms() - t0 < watchdog * 1000.0) usleep(10000);
      if (hipStreamQuery(c->stream) == hipErrorNotReady) {
        std::vector<unsigned> pg(4 * (size_t)(grid + 1));
        hipStream_t s2;
        (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
        (void)hipMemcpyAsync(pg.data(), fa.prog, 4 * pg.size(), hipMemcpyDeviceToHost, s2);
        (void)hipStreamSynchronize(s2);
        fprintf(stderr, "nwk watchdog: launch still running after %d s; wave markers:\n", watchdog);
        for (size_t q = 0; q < pg.size(); ++q)
          if (pg[q]) fprintf(stderr, "  wave %zu: %08x\n", q, pg[q]);
        fflush(stderr);
        _exit(3);
      }
    }
    unsigned herr = 0;
    HIP_TRY(hipMemcpyAsync(&herr, fa.err, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_oplen[par].p, fa.oplen, sizeof(int) * np, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_endij[par].p, fa.endij, sizeof(int2) * np, hipMemcpyDeviceToHost, c->stream));
    if (windowed || guard)
      HIP_TRY(hipMemcpyAsync(c->h_retry.p, fa.retry, sizeof(int) * np, hipMemcpyDeviceToHost, c->stream));
    if (guard) HIP_TRY(hipMemcpyAsync(c->h_endv[par].p, fa.endv, sizeof(int) * np, hipMemcpyDeviceToHost, c->stream));
    if (fuse) {
      // records arrive in host memory on their own
    } else if (devhash) {  // 68 bytes per pair instead of the move strings
      if ((rc = c->h_pen[par].ensure(4 * (size_t)np)) != NWK_OK) return rc;
      if ((rc = c->h_hash[par].ensure(64 * (size_t)np)) != NWK_OK) return rc;
      HIP_TRY(hipMemcpyAsync(c->h_pen[par].p, c->d_pen.p, 4 * (size_t)np, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipMemcpyAsync(c->h_hash[par].p, c->d_hash.p, 64 * (size_t)np, hipMemcpyDeviceToHost, c->stream));
    } else if (!hstream) {
      HIP_TRY(hipMemcpyAsync(c->h_ops[par].p, c->d_work.as<uint8_t>() + ops_base_b, (size_t)ops,
                             hipMemcpyDeviceToHost, c->stream));
    }
    const double tb1 = now_ms();
    HIP_TRY(hipStreamSynchronize(c->stream));
    const double tb2 = now_ms();
    if (herr) {
      std::vector<unsigned> dn((size_t)np);
      (void)hipMemcpy(dn.data(), c->d_done.p, sizeof(unsigned) * np, hipMemcpyDeviceToHost);
      unsigned cnt = 0;
      (void)hipMemcpy(&cnt, fa.counter, 4, hipMemcpyDeviceToHost);
      std::vector<int> olv((size_t)np);
      (void)hipMemcpy(olv.data(), c->d_oplen.p, sizeof(int) * np, hipMemcpyDeviceToHost);
      std::string d;
      for (int q = 0; q < np && q < 40; ++q)
        d += " " + std::to_string(dn[q]) + "/" + std::to_string(pd[q].nbands) + ":" + std::to_string(olv[q]);
      return fail(NWK_EKERNEL, "kernel hand-off timed out (err=%u); dequeued %u of %lld; done%s",
                  herr, cnt, (long long)ntasks, d.c_str());
    }
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[2]));
    st.fill_ms += ms;  // fill + fused traceback (one launch)
    float ms2 = 0;
    HIP_TRY(hipEventElapsedTime(&ms2, c->ev[2], c->ev[1]));
    st.traceback_ms += ms2;  // after the fill: segment gather (kPacked2) + device finalize (nw_rows, nw_hash)
    if (fa.stamps) {  // per-pair timeline (100 MHz ticks), relative to the earliest fill-done
      std::vector<unsigned long long> sp(13 * (size_t)np + 1);
      HIP_TRY(hipMemcpy(sp.data(), fa.stamps, 104 * (size_t)np + 8, hipMemcpyDeviceToHost));
      unsigned long long t0 = ~0ull, tlast = 0;
      for (int q = 0; q < np; ++q) t0 = std::min(t0, sp[8 * q]), tlast = std::max(tlast, sp[8 * q]);
      const unsigned long long tk0 = sp[11 * (size_t)np];
      fprintf(stderr, "nwk timeline: first pair filled %.3f ms, last pair filled %.3f ms after the kernel's first dequeue\n",
              (t0 - tk0) / 1e5, (tlast - tk0) / 1e5);
      if (segmented(pl.mode)) {
        fprintf(stderr, "nwk timeline: latest segment end per pair (ms after first dequeue; segment task.guess, moves):");
        for (int q = 0; q < np; ++q) {
          const unsigned long long te = sp[11 * (size_t)np + 1 + 2 * q], id = sp[11 * (size_t)np + 2 + 2 * q];
          const int sg = (int)(id >> 32), ng = std::max(1, pd[q].nguess);
          if (te) fprintf(stderr, " %d:%.2f(t%d.%d,%u)", q, (te - tk0) / 1e5, sg / ng, sg % ng, (unsigned)id);
        }
        fprintf(stderr, "\n");
      }
      fprintf(stderr, "nwk timeline (ms after first pair filled; kernel %.3f ms): pair m x n: filled -> traced | "
                      "trace cycles, runs, moves, tiles/(demand batches << 16 | ahead batches) | fill band-cycles, %% waiting on band above\n", ms);
      double bc = 0, wc = 0;
      for (int q = 0; q < np; ++q) {
        const unsigned long long* x = &sp[8 * q];
        bc += (double)x[6];
        wc += (double)x[7];
        fprintf(stderr, "  %3d %6d x %6d: %8.3f -> %8.3f (trace %.3f) | %.3g %.3g %llu %llu/%llu | %.3g %.1f%%\n", q,
                pd[q].m, pd[q].n, (x[0] - t0) / 1e5, (x[1] - t0) / 1e5, (x[1] - x[0]) / 1e5, (double)x[2], (double)x[3],
                x[4], x[5] >> 32, x[5] & 0xffffffffull, (double)x[6], x[6] ? 100.0 * (double)x[7] / (double)x[6] : 0.0);
      }
      if (segmented(pl.mode) && getenv("NWK_SEGDUMP")) {  // segment outcomes of the pairs traced last
        std::vector<int> si((size_t)nsegs * 8);
        HIP_TRY(hipMemcpy(si.data(), fa.seginfo, si.size() * 4, hipMemcpyDeviceToHost));
        std::vector<int> ord(np);
        for (int q = 0; q < np; ++q) ord[q] = q;
        std::sort(ord.begin(), ord.end(), [&](int x, int y) { return sp[8 * x + 1] > sp[8 * y + 1]; });
        for (int z = 0; z < std::min(np, 4); ++z) {
          const int q = ord[z];
          const int nt = (int)tasks_of(pl.mode, pd[q].nbands);
          fprintf(stderr, "segments of pair %d (%d x %d, spec every %d):", q, pd[q].m, pd[q].n, pd[q].spec_every);
          for (int b = 0; b < nt * pd[q].nguess; ++b) {
            const int* x = &si[8 * ((size_t)pd[q].seg_off + b)];
            if (x[0] || b == (nt - 1) * pd[q].nguess)
              fprintf(stderr, " [t%d.%d len %d end (%d,%d) -> %d@%d]", b / pd[q].nguess, b % pd[q].nguess, x[0], x[1], x[2], x[3], x[4]);
          }
          fprintf(stderr, "\n");
        }
        for (int q = 0; q < np; ++q) {  // the resolved chain of every pair
          const int nt = (int)tasks_of(pl.mode, pd[q].nbands), ng = pd[q].nguess;
          int sgi = (nt - 1) * ng, from = 0;
          fprintf(stderr, "chain of pair %d:", q);
          for (int hop = 0; hop < 64; ++hop) {
            const int* x = &si[8 * ((size_t)pd[q].seg_off + sgi)];
            fprintf(stderr, " t%d.%d[%d..%d)", sgi / ng, sgi % ng, from, x[0]);
            if (x[3] < 0) break;
            from = x[4];
            sgi = x[3];
          }
          fprintf(stderr, "\n");
        }
      }
      double w0 = 0, nw = 0, nsb = 0;
      for (int q = 0; q < np; ++q) {
        w0 += (double)sp[8 * (size_t)np + 3 * q];
        nw += (double)sp[8 * (size_t)np + 3 * q + 1];
        nsb += (double)sp[8 * (size_t)np + 3 * q + 2];
      }
      fprintf(stderr, "  all bands: %.4g cycles, %.1f%% waiting on the band above (%.1f%% before the first chunk); "
                      "%.4g waits over %.4g super-blocks\n",
              bc, bc > 0 ? 100.0 * wc / bc : 0.0, bc > 0 ? 100.0 * w0 / bc : 0.0, nw, nsb);
    }
    st.matrix_bytes += mat * 4;
    st.batches += 1;
    st.fill_launches += 1;
    // kBits windowed storage: pairs whose path left the window get no result
    // from this batch; they re-run with full storage in a later batch
    std::vector<char> skip;
    if (windowed || guard) {
      const int* rt = c->h_retry.as<int>();
      for (int q = 0; q < np; ++q) {
        if (!rt[q]) continue;
        if (skip.empty()) skip.assign((size_t)np, 0);
        skip[q] = 1;
        PairWork w = dp[pos + q];
        if (rt[q] == 2) {  // the guard, on the device (nw_rows / the fused finalize)
          const int ev = c->h_endv[par].as<int>()[q];
          const int pw = devhash && !fuse ? c->h_pen[par].as<int>()[q] : INT_MIN;  // (fused: on the device only)
          if ((rc = guard_rerun(c, &w, ev, pw, &st)) != NWK_OK) return rc;
        } else {
          st.window_retries += 1;
        }
        if ((rc = requeue(w)) != NWK_OK) return rc;
      }
    }
    if (fuse || hstream) {  // the consumer finishes on its own; the next join collects it
      fsync->skip = skip;
      fsync->done.store(1, std::memory_order_release);
      h_setup += tb1 - tb0;
      h_sync += tb2 - tb1;
      fused_all.push_back(fsync);
      if (end >= dp.size()) {
        const double tf0 = now_ms();
        fin.join();
        h_last += now_ms() - tf0;
      }
      pos = end;
      continue;
    }
    // ---- host finalize, overlapped with the next batch's kernel: it runs on
    // its own thread over this batch's host buffer set while the loop goes
    // on to set up, launch and wait for batch b+1 (buffer set par ^ 1).
    const double tj0 = now_ms();
    fin.join();
    h_join += now_ms() - tj0;
    const int* ol = c->h_oplen[par].as<int>();
    const int2* ej = c->h_endij[par].as<int2>();
    const uint8_t* hops = c->h_ops[par].as<uint8_t>();
    const PairWork* dw = dp.data() + pos;
    const int* hpen = c->h_pen[par].as<int>();
    const uint8_t* hhash = c->h_hash[par].as<uint8_t>();
    const int* hev = guard ? c->h_endv[par].as<int>() : nullptr;  // the fill's H(m, n) per slot
    GuardLog* glog = &gl;
    const int64_t gpos = (int64_t)pos;
    auto job = [c, a1, a2, np, dw, pd, ol, ej, hops, ops_base_b, sc, penalties, hashes, chain, devhash, hpen, hhash,
                skip, hev, glog, gpos]() mutable {
      // (guard: pairs whose walked path does not cost the fill's H(m, n) join the skipped ones and re-run)
      if (hev && !devhash && skip.empty()) skip.assign((size_t)np, 0);
      auto skipped = [&](int64_t q) { return !skip.empty() && skip[(size_t)q]; };
      if (devhash) {
        for (int64_t q = 0; q < np; ++q) {
          if (skipped(q)) continue;
          penalties[dw[q].out] = hpen[q];
          memcpy(hashes + 64 * dw[q].out, hhash + 64 * q, 64);
        }
      } else parallel_for(a1 ? 1 : c->host_threads, np, [&](int64_t q) {
        if (skipped(q)) return;
        const PairWork& w = dw[q];
        const PairDesc& d = pd[q];
        Finalized f;
        finalize_pair(c->seqs.data() + c->off[w.i], w.m, c->seqs.data() + c->off[w.j], w.n, sc,
                      hops + (d.ops_off - ops_base_b), ol[q], ej[q].x, ej[q].y, &f, a1, a2);
        if (hev && f.penalty != hev[q]) {
          glog->add(gpos + q, hev[q], f.penalty);
          skip[(size_t)q] = 1;  // (one thread per q: no other writer of this byte)
          return;
        }
        penalties[w.out] = f.penalty;
        memcpy(hashes + 64 * w.out, f.hash, 64);
      });
      for (int64_t q = 0; q < np; ++q)
        if (!skipped(q)) mark_ready(c, dw[q].out);
      if (chain) {  // serial: jobs never overlap each other (fin.join() before the next starts)
        parallel_for(c->host_threads, (np + 255) / 256, [&](int64_t b) {  // second-block schedules, in parallel
          for (int64_t q = b * 256; q < std::min<int64_t>(np, (b + 1) * 256); ++q)
            if (!skipped(q)) chain->prepare(dw[q].out);
        });
        for (int64_t q = 0; q < np; ++q)
          if (!skipped(q)) chain->ready[dw[q].out] = 1;
        chain->advance();
      }
    };
    if (end < dp.size()) fin.start(job);
    else { const double tf0 = now_ms(); job(); h_last += now_ms() - tf0; }
    h_setup += tb1 - tb0;
    h_sync += tb2 - tb1;
    pos = end;
  }
  fin.join();
  // pairs the host finalize rejected (fill-vs-walk guard) re-run in new batches
  const auto gbad = gl.take();
  if (gbad.empty()) break;
  for (const auto& g : gbad) {
    PairWork w = dp[(size_t)g.idx];
    if ((rc = guard_rerun(c, &w, g.endv, g.cost, &st)) != NWK_OK) return rc;
    if ((rc = requeue(w)) != NWK_OK) return rc;
  }
  }
  for (const auto& f : fused_all)
    if (f->missing) return fail(NWK_EKERNEL, "fused finalize: %lld pair(s) without a record", (long long)f->missing);
  st.total_ms = now_ms() - t_start;
  if (c->opts.verbose)
    fprintf(stderr, "nwk host: setup+launch %.3f ms, kernel+copies wait %.3f ms, finalize join %.3f ms, last finalize %.3f ms\n", h_setup, h_sync, h_join, h_last);
  c->stats = st;
  if (c->opts.verbose)
    fprintf(stderr, "nwk: %zu pairs, %.3g cells, fill %.3f ms (%.1f GCUPS), traceback %.3f ms, total %.3f ms, bits %d mode %d, %d batch(es), window %d, %d retries\n",
            work.size(), st.cells, st.fill_ms, st.fill_ms > 0 ? st.cells / st.fill_ms / 1e6 : 0.0,
            st.traceback_ms, st.total_ms, st.bits, st.mode, st.batches, dp.empty() ? 0 : dp[0].bits_w, (int)st.window_retries);
  return NWK_OK;
}

int make_work(const nwk_ctx* c, const int64_t* ids, int64_t n, std::vector<PairWork>* out) {
  const int64_t P = (int64_t)c->k * (c->k - 1) / 2;
  out->clear();
  out->reserve((size_t)n);
  for (int64_t q = 0; q < n; ++q) {
    if (ids[q] < 0 || ids[q] >= P) return fail(NWK_EINVAL, "pair id %lld out of range [0,%lld)", (long long)ids[q], (long long)P);
    PairWork w{};
    w.id = ids[q];
    w.out = q;
    pair_ij(ids[q], &w.i, &w.j);
    w.m = (int)(c->off[w.i + 1] - c->off[w.i]);
    w.n = (int)(c->off[w.j + 1] - c->off[w.j]);
    out->push_back(w);
  }
  return NWK_OK;
}

}  // namespace

extern "C" {

static int align_pairs_sc(nwk_ctx* c, const int64_t* pair_ids, int64_t npairs, const Scoring& sc,
                          int32_t* penalties, uint8_t* problem_hash) {
  if (!c || npairs < 0 || (npairs > 0 && (!pair_ids || !penalties || !problem_hash)))
    return fail(NWK_EINVAL, "nwk_align_pairs: bad argument");
  std::vector<PairWork> w;
  int rc = make_work(c, pair_ids, npairs, &w);
  if (rc != NWK_OK) return rc;
  return align_work(c, w, sc, penalties, problem_hash, nullptr, nullptr);
}

int nwk_align_pairs(nwk_ctx* c, const int64_t* pair_ids, int64_t npairs, int32_t pxy, int32_t pgap,
                    int32_t* penalties, uint8_t* problem_hash) {
  return align_pairs_sc(c, pair_ids, npairs, Scoring{pxy, pgap, false, 0, 0}, penalties, problem_hash);
}

int nwk_align_pairs_begin(nwk_ctx* c, const int64_t* pair_ids, int64_t npairs, int32_t pxy, int32_t pgap) {
  if (!c || npairs < 0 || (npairs > 0 && !pair_ids)) return fail(NWK_EINVAL, "nwk_align_pairs_begin: bad argument");
  if (c->pending) return fail(NWK_EINVAL, "nwk_align_pairs_begin: a call is already in flight on this context");
  c->a_ids.assign(pair_ids, pair_ids + npairs);
  c->a_pen.assign((size_t)std::max<int64_t>(npairs, 1), 0);
  c->a_hash.assign((size_t)std::max<int64_t>(npairs, 1) * 64, 0);
  c->pending = true;
  c->a_rc = NWK_OK;
  c->a_err.clear();
  c->a_ready.reset(new std::atomic<uint8_t>[(size_t)std::max<int64_t>(npairs, 1)]);
  for (int64_t q = 0; q < std::max<int64_t>(npairs, 1); ++q) c->a_ready[q].store(0, std::memory_order_relaxed);
  c->a_finished.store(0);
  c->async = std::thread([c, pxy, pgap]() {
    c->ready_out = c->a_ready.get();
    c->a_rc = nwk_align_pairs(c, c->a_ids.data(), (int64_t)c->a_ids.size(), pxy, pgap, c->a_pen.data(),
                              c->a_hash.data());
    c->ready_out = nullptr;
    if (c->a_rc != NWK_OK) c->a_err = g_err;
    c->a_finished.store(1, std::memory_order_release);
  });
  return NWK_OK;
}

int nwk_align_pairs_poll(nwk_ctx* c, int64_t from, int32_t* penalties, uint8_t* problem_hash, int64_t* upto) {
  if (!c || !c->pending || !upto || from < 0) return fail(NWK_EINVAL, "nwk_align_pairs_poll: bad argument");
  const int64_t n = (int64_t)c->a_ids.size();
  if (from > n) return fail(NWK_EINVAL, "nwk_align_pairs_poll: from %lld > %lld pairs", (long long)from, (long long)n);
  if (from < n && (!penalties || !problem_hash)) return fail(NWK_EINVAL, "nwk_align_pairs_poll: bad argument");
  const bool finished = c->a_finished.load(std::memory_order_acquire) != 0;
  int64_t q = from;
  while (q < n && c->a_ready[q].load(std::memory_order_acquire)) ++q;
  if (q > from) {
    memcpy(penalties + from, c->a_pen.data() + from, 4 * (size_t)(q - from));
    memcpy(problem_hash + 64 * from, c->a_hash.data() + 64 * from, 64 * (size_t)(q - from));
  }
  *upto = q;
  // a call that ended without every result: its error (nwk_align_pairs_end reports it too)
  if (finished && q < n && c->a_rc != NWK_OK) return fail(c->a_rc, "%s", c->a_err.c_str());
  return NWK_OK;
}

int nwk_align_pairs_end(nwk_ctx* c, int32_t* penalties, uint8_t* problem_hash) {
  if (!c || !c->pending) return fail(NWK_EINVAL, "nwk_align_pairs_end: no call in flight");
  c->async.join();
  c->pending = false;
  if (c->a_rc != NWK_OK) return fail(c->a_rc, "%s", c->a_err.c_str());
  const size_t n = c->a_ids.size();
  if (n && (!penalties || !problem_hash)) return fail(NWK_EINVAL, "nwk_align_pairs_end: bad argument");
  if (n) {
    memcpy(penalties, c->a_pen.data(), 4 * n);
    memcpy(problem_hash, c->a_hash.data(), 64 * n);
  }
  return NWK_OK;
}

int nwk_align_pairs_affine(nwk_ctx* c, const int64_t* pair_ids, int64_t npairs, int32_t pxy, int32_t go,
                           int32_t ge, int32_t* penalties, uint8_t* problem_hash) {
  return align_pairs_sc(c, pair_ids, npairs, Scoring{pxy, 0, true, go, ge}, penalties, problem_hash);
}

static int align_all_sc(nwk_ctx* c, const Scoring& sc, int32_t* penalties, uint8_t* problem_hash, char* hash_hex) {
  if (!c || !hash_hex) return fail(NWK_EINVAL, "nwk_align_all: bad argument");
  const int64_t P = (int64_t)c->k * (c->k - 1) / 2;
  if (P > 0 && !penalties) return fail(NWK_EINVAL, "nwk_align_all: penalties is NULL");
  std::vector<uint8_t> own;
  if (!problem_hash) {
    own.resize((size_t)std::max<int64_t>(P, 1) * 64);
    problem_hash = own.data();
  }
  std::vector<int64_t> ids((size_t)P);
  for (int64_t p = 0; p < P; ++p) ids[p] = p;
  std::vector<PairWork> w;
  int rc = make_work(c, ids.data(), P, &w);
  if (rc != NWK_OK) return rc;
  Chain ch;
  ch.init(problem_hash, P);
  if ((rc = align_work(c, w, sc, penalties, problem_hash, nullptr, nullptr, &ch)) != NWK_OK) return rc;
  ch.advance();  // pairs with no DP cells, if they are the tail
  if (ch.next != P) return fail(NWK_EKERNEL, "nwk_align_all: chain stopped at pair %lld of %lld", (long long)ch.next, (long long)P);
  ch.hex(hash_hex);
  return NWK_OK;
}

int nwk_align_all(nwk_ctx* c, int32_t pxy, int32_t pgap, int32_t* penalties, uint8_t* problem_hash, char* hash_hex) {
  return align_all_sc(c, Scoring{pxy, pgap, false, 0, 0}, penalties, problem_hash, hash_hex);
}

int nwk_align_all_affine(nwk_ctx* c, int32_t pxy, int32_t go, int32_t ge, int32_t* penalties, uint8_t* problem_hash,
                         char* hash_hex) {
  return align_all_sc(c, Scoring{pxy, 0, true, go, ge}, penalties, problem_hash, hash_hex);
}

int nwk_last_stats(const nwk_ctx* c, nwk_stats* out) {
  if (!c || !out) return fail(NWK_EINVAL, "nwk_last_stats: bad argument");
  *out = c->stats;
  return NWK_OK;
}

static int min_penalty_sc(nwk_ctx* c, const uint8_t* x, int32_t m, const uint8_t* y, int32_t n, const Scoring& sc,
                          uint8_t* a1, uint8_t* a2, int32_t* alen, int32_t* penalty) {
  if (!c || m < 0 || n < 0 || (m && !x) || (n && !y) || !a1 || !a2 || !alen || !penalty)
    return fail(NWK_EINVAL, "nwk_get_minimum_penalty: bad argument");
  // set {y, x}: pair 0 = (i=1 -> rows x, j=0 -> columns y)
  std::vector<uint8_t> s((size_t)m + n);
  if (n) memcpy(s.data(), y, (size_t)n);
  if (m) memcpy(s.data() + n, x, (size_t)m);
  const int64_t off[3] = {0, n, (int64_t)n + m};
  int rc = nwk_set_sequences(c, s.data(), off, 2);
  if (rc != NWK_OK) return rc;
  std::vector<PairWork> w;
  const int64_t id = 0;
  if ((rc = make_work(c, &id, 1, &w)) != NWK_OK) return rc;
  std::vector<uint8_t> r1, r2;
  unsigned char h[64];
  if ((rc = align_work(c, w, sc, penalty, h, &r1, &r2)) != NWK_OK) return rc;
  memcpy(a1, r1.data(), r1.size());
  memcpy(a2, r2.data(), r2.size());
  *alen = (int32_t)r1.size();
  return NWK_OK;
}

int nwk_get_minimum_penalty(nwk_ctx* c, const uint8_t* x, int32_t m, const uint8_t* y, int32_t n, int32_t pxy,
                            int32_t pgap, uint8_t* a1, uint8_t* a2, int32_t* alen, int32_t* penalty) {
  return min_penalty_sc(c, x, m, y, n, Scoring{pxy, pgap, false, 0, 0}, a1, a2, alen, penalty);
}

int nwk_get_minimum_penalty_affine(nwk_ctx* c, const uint8_t* x, int32_t m, const uint8_t* y, int32_t n, int32_t pxy,
                                   int32_t go, int32_t ge, uint8_t* a1, uint8_t* a2, int32_t* alen, int32_t* penalty) {
  return min_penalty_sc(c, x, m, y, n, Scoring{pxy, 0, true, go, ge}, a1, a2, alen, penalty);
}

int nwk_shard_pairs(const int64_t* offsets, int32_t k, int32_t rank, int32_t world, int64_t* out_ids,
                    int64_t* out_n) {
  if (!offsets || k < 0 || world < 1 || rank < 0 || rank >= world || !out_n)
    return fail(NWK_EINVAL, "nwk_shard_pairs: bad argument");
  const int64_t P = (int64_t)k * (k - 1) / 2;
  std::vector<std::pair<double, int64_t>> cost((size_t)P);
  int64_t p = 0;
  for (int i = 1; i < k; ++i)
    for (int j = 0; j < i; ++j, ++p)
      cost[p] = {(double)(offsets[i + 1] - offsets[i]) * (double)(offsets[j + 1] - offsets[j]) + 1.0, p};
  std::sort(cost.begin(), cost.end(), [](const auto& a, const auto& b) {
    return a.first != b.first ? a.first > b.first : a.second < b.second;
  });
  std::vector<double> load((size_t)world, 0.0);
  int64_t cnt = 0;
  for (const auto& cp : cost) {
    int best = 0;
    for (int r = 1; r < world; ++r)
      if (load[r] < load[best]) best = r;
    load[best] += cp.first;
    if (best == rank) {
      if (out_ids) out_ids[cnt] = cp.second;
      ++cnt;
    }
  }
  if (out_ids) std::sort(out_ids, out_ids + cnt);
  *out_n = cnt;
  return NWK_OK;
}

int nwk_finalize_moves(const uint8_t* x, int32_t m, const uint8_t* y, int32_t n, int32_t pxy, int32_t pgap,
                       const uint8_t* moves, int64_t nmoves, uint8_t* a1, uint8_t* a2, int32_t* alen,
                       int32_t* penalty, uint8_t* problem_hash) {
  if (m < 0 || n < 0 || nmoves < 0 || (m > 0 && !x) || (n > 0 && !y) || (nmoves > 0 && !moves) || !alen ||
      !penalty || !problem_hash || ((m > 0 || n > 0) && (!a1 || !a2)))
    return fail(NWK_EINVAL, "nwk_finalize_moves: bad argument");
  // walk the moves from (m, n) to where they end, which must be a border cell
  int64_t i = m, j = n;
  for (int64_t t = 0; t < nmoves; ++t) {
    const uint8_t op = moves[t];
    if (op != 'D' && op != 'U' && op != 'L') return fail(NWK_EINVAL, "nwk_finalize_moves: move %lld is not D/U/L", (long long)t);
    if (i == 0 || j == 0) return fail(NWK_EINVAL, "nwk_finalize_moves: move %lld leaves the border", (long long)t);
    i -= op != 'L';
    j -= op != 'U';
  }
  if (i != 0 && j != 0) return fail(NWK_EINVAL, "nwk_finalize_moves: walk ends at (%lld, %lld), off the border", (long long)i, (long long)j);
  // walk order from (m, n) is the order the kernels emit and finalize_pair takes
  std::vector<uint8_t> r1, r2;
  Finalized f;
  finalize_pair(x, m, y, n, Scoring{pxy, pgap, false, 0, 0}, moves, (int)nmoves, (int)i, (int)j, &f, &r1, &r2);
  if (!r1.empty()) {
    memcpy(a1, r1.data(), r1.size());
    memcpy(a2, r2.data(), r2.size());
  }
  *alen = (int32_t)r1.size();
  *penalty = f.penalty;
  memcpy(problem_hash, f.hash, 64);
  return NWK_OK;
}

int nwk_chain_hash(const uint8_t* ph, int64_t P, char* hash_hex) {
  if (!hash_hex || (P > 0 && !ph)) return fail(NWK_EINVAL, "nwk_chain_hash: bad argument");
  Chain ch;
  ch.init(ph, std::max<int64_t>(P, 0));
  unsigned hc = std::thread::hardware_concurrency();
  parallel_for((int)std::min(16u, hc ? hc : 1u), (P + 1023) / 1024, [&](int64_t b) {
    for (int64_t p = b * 1024; p < std::min(P, (b + 1) * 1024); ++p) ch.prepare(p);
  });
  std::fill(ch.ready.begin(), ch.ready.end(), 1);
  ch.advance();
  ch.hex(hash_hex);
  return NWK_OK;
}

// Streaming chain (skel:159 as results arrive, sub:305-337's collect-then-chain
// overlapped): feed() stores records and computes their second-block schedules
// on the caller's thread; a worker thread advances the chain over the ready
// prefix of canonical ids while the caller goes on (e.g. aligning the next
// chunk of its shard).
}  // extern "C"

struct nwk_chain {
  int64_t P = 0;
  std::vector<uint8_t> ph;       // [P][64]
  std::vector<uint64_t> kw;      // [P][80] second-block schedules
  std::vector<int32_t> pen;      // [P]
  std::unique_ptr<std::atomic<char>[]> ready;
  std::atomic<int64_t> fed{0};
  int64_t next = 0;              // worker-owned
  ChainAcc acc;
  std::mutex mu;
  std::condition_variable cv;
  bool closed = false;
  std::thread worker;
  void run() {
    for (;;) {
      while (next < P && ready[next].load(std::memory_order_acquire)) {
        chain_step(&acc, kw.data() + 80 * next);
        ++next;
      }
      std::unique_lock<std::mutex> lk(mu);
      if (next >= P) return;
      if (ready[next].load(std::memory_order_acquire)) continue;
      if (closed) return;
      cv.wait(lk);
    }
  }
};

extern "C" {

int nwk_chain_create(int64_t P, nwk_chain** out) {
  if (!out || P < 0) return fail(NWK_EINVAL, "nwk_chain_create: bad argument");
  std::unique_ptr<nwk_chain> ch(new nwk_chain);
  ch->P = P;
  ch->ph.assign((size_t)P * 64, 0);
  ch->kw.assign((size_t)P * 80, 0);
  ch->pen.assign((size_t)P, 0);
  ch->ready.reset(new std::atomic<char>[(size_t)std::max<int64_t>(P, 1)]);
  for (int64_t p = 0; p < P; ++p) ch->ready[p].store(0, std::memory_order_relaxed);
  nwk_chain* c = ch.get();
  ch->worker = std::thread([c]() { c->run(); });
  *out = ch.release();
  return NWK_OK;
}

int nwk_chain_feed(nwk_chain* ch, const int64_t* ids, const int32_t* penalties, const uint8_t* problem_hash,
                   int64_t n) {
  if (!ch || n < 0 || (n > 0 && (!ids || !problem_hash))) return fail(NWK_EINVAL, "nwk_chain_feed: bad argument");
  // each id once: against earlier calls (ready) and within this batch (seen)
  std::unordered_set<int64_t> seen;
  seen.reserve((size_t)n);
  for (int64_t q = 0; q < n; ++q)
    if (ids[q] < 0 || ids[q] >= ch->P || ch->ready[ids[q]].load(std::memory_order_relaxed) || !seen.insert(ids[q]).second)
      return fail(NWK_EINVAL, "nwk_chain_feed: pair id %lld out of range or fed twice", (long long)ids[q]);
  for (int64_t q = 0; q < n; ++q) {
    const int64_t p = ids[q];
    memcpy(ch->ph.data() + 64 * p, problem_hash + 64 * q, 64);
    if (penalties) ch->pen[p] = penalties[q];
    chain_schedule(problem_hash + 64 * q, ch->kw.data() + 80 * p);
    ch->ready[p].store(1, std::memory_order_release);
  }
  ch->fed += n;
  { std::lock_guard<std::mutex> lk(ch->mu); }
  ch->cv.notify_one();
  return NWK_OK;
}

int nwk_chain_finish(nwk_chain* ch, char* hash_hex, int32_t* penalties, uint8_t* problem_hash) {
  if (!ch || !hash_hex) return fail(NWK_EINVAL, "nwk_chain_finish: bad argument");
  {
    std::lock_guard<std::mutex> lk(ch->mu);
    ch->closed = true;
  }
  ch->cv.notify_one();
  if (ch->worker.joinable()) ch->worker.join();
  if (ch->next != ch->P)
    return fail(NWK_EINVAL, "nwk_chain_finish: pair %lld of %lld was never fed", (long long)ch->next, (long long)ch->P);
  chain_hex(ch->acc, hash_hex);
  hash_hex[ch->acc.empty ? 0 : 128] = 0;
  if (penalties && ch->P) memcpy(penalties, ch->pen.data(), 4 * (size_t)ch->P);
  if (problem_hash && ch->P) memcpy(problem_hash, ch->ph.data(), 64 * (size_t)ch->P);
  return NWK_OK;
}

void nwk_chain_destroy(nwk_chain* ch) {
  if (!ch) return;
  {
    std::lock_guard<std::mutex> lk(ch->mu);
    ch->closed = true;
  }
  ch->cv.notify_one();
  if (ch->worker.joinable()) ch->worker.join();
  delete ch;
}

void nwk_sha512_hex(const uint8_t* data, int64_t len, char* out_hex) {
  sha512_hex(data, (size_t)len, out_hex);
  out_hex[128] = 0;
}

// ---------------------------------------------------------------------------
// getMinimumPenalties: single device, or G devices + one ncclAllGather.
// ---------------------------------------------------------------------------
struct ResultRecord {
  int32_t pair_id;
  int32_t penalty;
  uint8_t hash[64];
};
static_assert(sizeof(ResultRecord) == 72, "record layout");

static int min_penalties_sc(const uint8_t* seqs, const int64_t* offsets, int32_t k, const Scoring& sc,
                            int32_t* penalties, char* hash_hex, const nwk_opts* opts) {
  if (k < 0 || !hash_hex || (k > 0 && !offsets)) return fail(NWK_EINVAL, "nwk_get_minimum_penalties: bad argument");
  nwk_opts o;
  nwk_opts_default(&o);
  if (opts) o = *opts;
  const int64_t P = (int64_t)k * (k - 1) / 2;
  if (P > 0 && !penalties) return fail(NWK_EINVAL, "nwk_get_minimum_penalties: penalties is NULL");
  std::vector<uint8_t> ph((size_t)std::max<int64_t>(P, 1) * 64);
  const int G = std::max(1, o.ngpus);
  if (P == 0) {
    hash_hex[0] = 0;
    return NWK_OK;
  }
  if (G == 1 && !o.collective) {
    nwk_ctx* c = nullptr;
    int rc = nwk_ctx_create(&o, &c);
    if (rc != NWK_OK) return rc;
    rc = nwk_set_sequences(c, seqs, offsets, k);
    if (rc == NWK_OK) rc = align_all_sc(c, sc, penalties, ph.data(), hash_hex);
    nwk_ctx_destroy(c);
    return rc;
  }
  if (G > nwk_device_count()) return fail(NWK_EINVAL, "ngpus=%d > visible devices %d", G, nwk_device_count());
  // Shards: LPT on cell cost; every rank sends a padded block of `per` records.
  std::vector<std::vector<int64_t>> shard((size_t)G);
  int64_t per = 0;
  for (int r = 0; r < G; ++r) {
    int64_t n = 0;
    shard[r].resize((size_t)P);
    nwk_shard_pairs(offsets, k, r, G, shard[r].data(), &n);
    shard[r].resize((size_t)n);
    per = std::max(per, n);
  }
  std::vector<ncclComm_t> comms((size_t)G);
  std::vector<int> devs((size_t)G);
  for (int r = 0; r < G; ++r) devs[r] = r;
  if (ncclCommInitAll(comms.data(), G, devs.data()) != ncclSuccess)
    return fail(NWK_ECOMM, "ncclCommInitAll failed");
  std::vector<ResultRecord> gathered((size_t)per * G);
  // Collective buffers and streams for every rank are set up here, before any
  // rank thread starts: either all of them exist and every rank then calls
  // ncclAllGather exactly once (a rank whose alignment failed still joins with
  // records tagged -2), or none does and the call fails without a collective.
  // No rank can be left waiting in the all-gather for a peer that bailed out.
  std::vector<void*> dsend((size_t)G, nullptr), drecv((size_t)G, nullptr);
  std::vector<hipStream_t> cstream((size_t)G, nullptr);
  auto free_coll = [&]() {
    for (int r = 0; r < G; ++r) {
      (void)hipSetDevice(r);
      if (dsend[r]) (void)hipFree(dsend[r]);
      if (drecv[r]) (void)hipFree(drecv[r]);
      if (cstream[r]) (void)hipStreamDestroy(cstream[r]);
    }
    for (auto& cm : comms) ncclCommDestroy(cm);
  };
  for (int r = 0; r < G; ++r) {
    if (hipSetDevice(r) != hipSuccess || hipMalloc(&dsend[r], sizeof(ResultRecord) * per) != hipSuccess ||
        hipMalloc(&drecv[r], sizeof(ResultRecord) * per * G) != hipSuccess ||
        hipStreamCreateWithFlags(&cstream[r], hipStreamNonBlocking) != hipSuccess) {
      free_coll();
      return fail(NWK_ENOMEM, "rank %d: collective buffers could not be allocated", r);
    }
  }
  std::vector<int> rcs((size_t)G, NWK_OK);
  std::vector<std::string> errs((size_t)G);
  std::vector<std::thread> th;
  for (int r = 0; r < G; ++r) {
    th.emplace_back([&, r]() {
      nwk_opts ro = o;
      ro.device = r;
      nwk_ctx* c = nullptr;
      int rc = nwk_ctx_create(&ro, &c);
      const int64_t n = (int64_t)shard[r].size();
      std::vector<ResultRecord> rec((size_t)per);
      for (auto& x : rec) x.pair_id = -1;
      if (rc == NWK_OK) rc = nwk_set_sequences(c, seqs, offsets, k);
      std::vector<int32_t> pen((size_t)std::max<int64_t>(n, 1));
      std::vector<uint8_t> hh((size_t)std::max<int64_t>(n, 1) * 64);
      if (rc == NWK_OK && n > 0) rc = align_pairs_sc(c, shard[r].data(), n, sc, pen.data(), hh.data());
      for (int64_t q = 0; rc == NWK_OK && q < n; ++q) {
        rec[q].pair_id = (int32_t)shard[r][q];
        rec[q].penalty = pen[q];
        memcpy(rec[q].hash, hh.data() + 64 * q, 64);
      }
      // Every rank joins the collective exactly once, even after a local
      // failure (records tagged -2), so no peer is left waiting.
      if (rc != NWK_OK) {
        for (auto& x : rec) x.pair_id = -2;
        errs[r] = g_err;
      }
      (void)hipSetDevice(r);
      int crc = NWK_OK;
      if (hipMemcpy(dsend[r], rec.data(), sizeof(ResultRecord) * per, hipMemcpyHostToDevice) != hipSuccess)
        crc = NWK_EDEVICE;
      if (ncclAllGather(dsend[r], drecv[r], sizeof(ResultRecord) * per, ncclUint8, comms[r], cstream[r]) != ncclSuccess)
        crc = NWK_ECOMM;
      if (hipStreamSynchronize(cstream[r]) != hipSuccess) crc = NWK_ECOMM;
      if (r == 0 && crc == NWK_OK &&
          hipMemcpy(gathered.data(), drecv[r], sizeof(ResultRecord) * per * G, hipMemcpyDeviceToHost) != hipSuccess)
        crc = NWK_EDEVICE;
      rcs[r] = rc != NWK_OK ? rc : crc;
      if (c) nwk_ctx_destroy(c);
    });
  }
  for (auto& t : th) t.join();
  free_coll();
  for (int r = 0; r < G; ++r)
    if (rcs[r] != NWK_OK) return fail(rcs[r], "rank %d: %s", r, errs[r].empty() ? "collective failed" : errs[r].c_str());
  std::vector<char> have((size_t)P, 0);
  for (const auto& x : gathered) {
    if (x.pair_id < 0) continue;
    penalties[x.pair_id] = x.penalty;
    memcpy(ph.data() + 64 * (int64_t)x.pair_id, x.hash, 64);
    have[x.pair_id] = 1;
  }
  for (int64_t p = 0; p < P; ++p)
    if (!have[p]) return fail(NWK_ECOMM, "pair %lld missing after all-gather", (long long)p);
  return nwk_chain_hash(ph.data(), P, hash_hex);
}

// ---------------------------------------------------------------------------
// Multi-process communicator (nwk_comm_*): one RCCL rank per process.
// ---------------------------------------------------------------------------
struct nwk_comm {
  int device = 0, world = 0, rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  void* dbuf = nullptr;  // staging: send block | world x recv blocks
  size_t dcap = 0;
};

static_assert(sizeof(ncclUniqueId) <= NWK_COMM_ID_BYTES, "ncclUniqueId larger than NWK_COMM_ID_BYTES");

int nwk_comm_unique_id(uint8_t* id) {
  if (!id) return fail(NWK_EINVAL, "nwk_comm_unique_id: id is NULL");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return fail(NWK_ECOMM, "ncclGetUniqueId failed");
  memset(id, 0, NWK_COMM_ID_BYTES);
  memcpy(id, &u, sizeof(u));
  return NWK_OK;
}

int nwk_comm_create(int32_t device, const uint8_t* id, int32_t world, int32_t rank, nwk_comm** out) {
  if (!id || !out || world < 1 || rank < 0 || rank >= world) return fail(NWK_EINVAL, "nwk_comm_create: bad argument");
  *out = nullptr;
  if (device < 0 || device >= nwk_device_count()) return fail(NWK_EDEVICE, "nwk_comm_create: no device %d", device);
  auto* cm = new nwk_comm;
  cm->device = device;
  cm->world = world;
  cm->rank = rank;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&cm->stream, hipStreamNonBlocking) != hipSuccess) {
    delete cm;
    return fail(NWK_EDEVICE, "nwk_comm_create: device %d", device);
  }
  if (ncclCommInitRank(&cm->comm, world, u, rank) != ncclSuccess) {
    (void)hipStreamDestroy(cm->stream);
    delete cm;
    return fail(NWK_ECOMM, "ncclCommInitRank failed (rank %d of %d)", rank, world);
  }
  *out = cm;
  return NWK_OK;
}

static int comm_stage(nwk_comm* cm, size_t bytes) {
  if (bytes <= cm->dcap) return NWK_OK;
  if (cm->dbuf) (void)hipFree(cm->dbuf);
  cm->dbuf = nullptr;
  cm->dcap = 0;
  if (hipMalloc(&cm->dbuf, bytes) != hipSuccess) return fail(NWK_ENOMEM, "nwk_comm: staging buffer of %zu bytes", bytes);
  cm->dcap = bytes;
  return NWK_OK;
}

int nwk_comm_all_gather(nwk_comm* cm, const void* send, int64_t bytes, void* recv) {
  if (!cm || bytes < 0 || (bytes > 0 && (!send || !recv))) return fail(NWK_EINVAL, "nwk_comm_all_gather: bad argument");
  if (hipSetDevice(cm->device) != hipSuccess) return fail(NWK_EDEVICE, "nwk_comm_all_gather: device");
  const size_t b = (size_t)std::max<int64_t>(bytes, 1);
  int rc = comm_stage(cm, b * (size_t)(cm->world + 1));
  if (rc != NWK_OK) return rc;
  uint8_t* ds = static_cast<uint8_t*>(cm->dbuf);
  uint8_t* dr = ds + b;
  if (bytes > 0) HIP_TRY(hipMemcpyAsync(ds, send, (size_t)bytes, hipMemcpyHostToDevice, cm->stream));
  if (ncclAllGather(ds, dr, b, ncclUint8, cm->comm, cm->stream) != ncclSuccess)
    return fail(NWK_ECOMM, "ncclAllGather failed (rank %d)", cm->rank);
  if (bytes > 0) {
    if (b == (size_t)bytes) {
      HIP_TRY(hipMemcpyAsync(recv, dr, b * cm->world, hipMemcpyDeviceToHost, cm->stream));
    } else {
      for (int r = 0; r < cm->world; ++r)
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t*>(recv) + (size_t)bytes * r, dr + b * r, (size_t)bytes,
                               hipMemcpyDeviceToHost, cm->stream));
    }
  }
  HIP_TRY(hipStreamSynchronize(cm->stream));
  return NWK_OK;
}

int nwk_comm_all_reduce_max_f64(nwk_comm* cm, double* vals, int64_t n) {
  if (!cm || n < 1 || !vals) return fail(NWK_EINVAL, "nwk_comm_all_reduce_max_f64: bad argument");
  if (hipSetDevice(cm->device) != hipSuccess) return fail(NWK_EDEVICE, "nwk_comm_all_reduce_max_f64: device");
  int rc = comm_stage(cm, sizeof(double) * (size_t)n);
  if (rc != NWK_OK) return rc;
  HIP_TRY(hipMemcpyAsync(cm->dbuf, vals, sizeof(double) * n, hipMemcpyHostToDevice, cm->stream));
  if (ncclAllReduce(cm->dbuf, cm->dbuf, (size_t)n, ncclFloat64, ncclMax, cm->comm, cm->stream) != ncclSuccess)
    return fail(NWK_ECOMM, "ncclAllReduce failed (rank %d)", cm->rank);
  HIP_TRY(hipMemcpyAsync(vals, cm->dbuf, sizeof(double) * n, hipMemcpyDeviceToHost, cm->stream));
  HIP_TRY(hipStreamSynchronize(cm->stream));
  return NWK_OK;
}

void nwk_comm_destroy(nwk_comm* cm) {
  if (!cm) return;
  (void)hipSetDevice(cm->device);
  if (cm->comm) ncclCommDestroy(cm->comm);
  if (cm->dbuf) (void)hipFree(cm->dbuf);
  if (cm->stream) (void)hipStreamDestroy(cm->stream);
  delete cm;
}

int nwk_device_synchronize(int32_t device) {
  if (device < 0 || device >= nwk_device_count()) return fail(NWK_EDEVICE, "nwk_device_synchronize: no device %d", device);
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipDeviceSynchronize());
  return NWK_OK;
}

// ---------------------------------------------------------------------------
// Progressive sum-of-pairs MSA (build-defined, oracle
// oracle/msa_oracle.c nwo_msa): UPGMA on the pairwise penalties, then one
// profile-profile DP per merge on the GPU (nw_profile + the fused affine-code
// traceback), merges of independent subtrees batched into one launch.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

struct Prof {
  std::vector<int> cnt;       // len x S column counts (S - 1 = gaps); freed once merged
  std::vector<int> up;        // column -> column of the merged profile (set by the merge)
  std::vector<int> members;   // input sequence index of each row
  int len = 0, parent = -1;
};

// Column symbol counts of a profile (S symbols, the last = gap).
// a leaf's column counts (merged profiles add their children's along the path)
void leaf_counts(const uint8_t* seq, int len, const uint8_t* code_of, int S, std::vector<int>* cnt) {
  cnt->assign((size_t)len * S, 0);
  for (int i = 0; i < len; ++i) (*cnt)[(size_t)i * S + code_of[seq[i]]]++;
}

// NWK_WATCHDOG=<s> debug: report the wave markers of a launch that does not finish, then exit.
void watchdog_wait(nwk_ctx* c, const unsigned* prog, int grid) {
  static const int watchdog = getenv("NWK_WATCHDOG") ? atoi(getenv("NWK_WATCHDOG")) : 0;
  if (watchdog <= 0 || !prog) return;
  const double t0 = now_ms();
  while (hipStreamQuery(c->stream) == hipErrorNotReady && now_ms() - t0 < watchdog * 1000.0) usleep(10000);
  if (hipStreamQuery(c->stream) != hipErrorNotReady) return;
  std::vector<unsigned> pg(4 * (size_t)(grid + 1));
  hipStream_t s2;
  (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  (void)hipMemcpyAsync(pg.data(), prog, 4 * pg.size(), hipMemcpyDeviceToHost, s2);
  (void)hipStreamSynchronize(s2);
  fprintf(stderr, "nwk watchdog: launch still running after %d s; wave markers:\n", watchdog);
  for (size_t q = 0; q < pg.size(); ++q)
    if (pg[q]) fprintf(stderr, "  wave %zu: %08x\n", q, pg[q]);
  fflush(stderr);
  _exit(3);
}

}  // namespace

extern "C" {

int nwk_msa(nwk_ctx* c, int32_t pxy, int32_t pgap, const int32_t* penalties, uint8_t* rows, int64_t cap,
            int64_t* len, int64_t* sop) {
  if (!c || !len || !sop || (c->k > 1 && !penalties) || (c->k > 0 && !rows)) return fail(NWK_EINVAL, "nwk_msa: bad argument");
  if (pxy < 0 || pgap < 0) return fail(NWK_EINVAL, "nwk_msa: penalties must be >= 0");
  if (c->has_us) return fail(NWK_EINVAL, "nwk_msa: '_' is the gap symbol and may not occur in the input");
  const int k = c->k, S = c->alpha + 1, gap = S - 1;
  if (S > kProfSyms) return fail(NWK_EINVAL, "nwk_msa: %d distinct input bytes (at most %d)", c->alpha, kProfSyms - 1);
  *len = 0;
  *sop = 0;
  // stats (nwk_last_stats): fill_ms = the nw_profile launches (HIP events), traceback_ms = 0 (the
  // walk runs inside them), cells = sum of merge DP cells, fill_launches = batches = tree levels
  const double t_start = now_ms();
  nwk_stats st{};
  st.mode = kProfileDP;
  st.bits = 4;
  c->stats = st;
  if (k == 0) return NWK_OK;
  const int nc = 2 * k - 1;
  std::vector<Prof> prof((size_t)nc);
  for (int s = 0; s < k; ++s) {
    prof[s].len = (int)(c->off[s + 1] - c->off[s]);
    leaf_counts(c->seqs.data() + c->off[s], prof[s].len, c->code_of, S, &prof[s].cnt);
    prof[s].members = {s};
  }
  // ---- UPGMA (oracle nwo_msa): mean pairwise penalty, exact ratio compare, ties -> smallest ids
  std::vector<int64_t> Ssum((size_t)nc * nc, 0);
  std::vector<int> sz((size_t)nc, 0), round_of((size_t)nc, 0);
  std::vector<char> alive((size_t)nc, 0);
  for (int s = 0; s < k; ++s) sz[s] = 1, alive[s] = 1;
  for (int i = 1; i < k; ++i)
    for (int j = 0; j < i; ++j) Ssum[(size_t)i * nc + j] = Ssum[(size_t)j * nc + i] = penalties[(int64_t)i * (i - 1) / 2 + j];
  struct Merge { int x, y, id; };
  std::vector<Merge> merges;
  for (int nid = k; nid < nc; ++nid) {
    int ba = -1, bb = -1;
    for (int a = 0; a < nid; ++a) {
      if (!alive[a]) continue;
      for (int b = a + 1; b < nid; ++b) {
        if (!alive[b]) continue;
        if (ba < 0) { ba = a; bb = b; continue; }
        const __int128 lhs = (__int128)Ssum[(size_t)a * nc + b] * sz[ba] * sz[bb];
        const __int128 rhs = (__int128)Ssum[(size_t)ba * nc + bb] * sz[a] * sz[b];
        if (lhs < rhs) { ba = a; bb = b; }
      }
    }
    merges.push_back(Merge{bb, ba, nid});  // rows: the younger cluster (skel's x = genes[i], i > j)
    sz[nid] = sz[ba] + sz[bb];
    round_of[nid] = 1 + std::max(round_of[ba], round_of[bb]);
    alive[ba] = alive[bb] = 0;
    alive[nid] = 1;
    for (int o = 0; o < nid; ++o)
      if (alive[o]) Ssum[(size_t)nid * nc + o] = Ssum[(size_t)o * nc + nid] = Ssum[(size_t)ba * nc + o] + Ssum[(size_t)bb * nc + o];
  }
  HIP_TRY(hipSetDevice(c->device));
  int rc;
  const int max_round = k > 1 ? round_of[nc - 1] : 0;
  DevBuf &d_prow = c->d_msa[0], &d_pcol = c->d_msa[1], &d_mw = c->d_msa[2], &d_pd = c->d_pairs, &d_tk = c->d_tasks;
  double t_lvl = now_ms(), t_mg = t_lvl, t_prep = 0, t_wait = 0, t_build = 0;  // (verbose >= 2: host phases per level)
  for (int rd = 1; rd <= max_round; ++rd) {
    std::vector<Merge> ms;
    for (const auto& m : merges)
      if (round_of[m.id] == rd) ms.push_back(m);
    const int np = (int)ms.size();
    // ---- profile arrays: X columns (DP rows) {rc[0..5], gx, H[i][0]}, Y columns {cnt[0..5], gy, H[0][j]}
    std::vector<int> hrow, hcol;
    std::vector<PairDesc> pd((size_t)np);
    std::vector<std::vector<int>> rc_host((size_t)np);
    int64_t mat = 0, bnd = 0, ops = 0, ntasks = 0, maxpk = 0;  // maxpk: largest rc / count (profile packing)
    for (int q = 0; q < np; ++q) {
      const Prof &X = prof[ms[q].x], &Y = prof[ms[q].y];
      const int nx = (int)X.members.size(), ny = (int)Y.members.size(), LX = X.len, LY = Y.len;
      const std::vector<int>& cx = X.cnt;
      const std::vector<int>& cyv = Y.cnt;
      int64_t maxstep = 0, acc = 0;
      maxpk = std::max<int64_t>(maxpk, std::max(nx, ny));  // (a column count is at most its profile's members)
      const int64_t xoff = (int64_t)hrow.size() / 8;
      std::vector<int>& rch = rc_host[q];
      rch.assign((size_t)LX * 8, 0);
      for (int i = 0; i < LX; ++i) {
        // rc[b] = sum_a cnt[a] c(a, b) in closed form (the SoP symbol costs: 0 on the
        // diagonal and gap vs gap, pxy between residues, pgap residue vs gap): with ng
        // residues and cg gaps in the column, rc[b] = pxy (ng - cnt[b]) + pgap cg for a
        // residue b, pgap ng for the gap
        const int* xc = &cx[(size_t)i * S];
        int64_t ng = 0;
        for (int a2 = 0; a2 < gap; ++a2) ng += xc[a2];
        int64_t rcb[kProfSyms] = {0};
        for (int b = 0; b < gap; ++b) rcb[b] = (int64_t)pxy * (ng - xc[b]) + (int64_t)pgap * xc[gap];
        rcb[gap] = (int64_t)pgap * ng;
        const int64_t gx = (int64_t)(nx - cx[(size_t)i * S + gap]) * ny * pgap;
        acc += gx;
        for (int b = 0; b < kProfSyms; ++b) rch[(size_t)i * 8 + b] = (int)(b < S ? rcb[b] : 0);
        rch[(size_t)i * 8 + 6] = (int)gx;
        rch[(size_t)i * 8 + 7] = (int)acc;
        int64_t mx = gx;
        for (int b = 0; b < S; ++b) mx = std::max(mx, rcb[b] * ny), maxpk = std::max(maxpk, rcb[b]);
        maxstep = std::max(maxstep, mx);
        if (mx >= (1 << 24)) return fail(NWK_EINVAL, "nwk_msa: profile costs exceed the kernel's 24-bit products");
      }
      hrow.insert(hrow.end(), rch.begin(), rch.end());
      // columns: entry y_off + j holds column j (j = 0: H[0][0] = 0), 64 pad entries before, 192 after
      const int64_t yoff = (int64_t)hcol.size() / 8 + 64;
      std::vector<int> colv((size_t)(LY + 64 + 192) * 8, 0);
      int64_t accy = 0;
      for (int j = 1; j <= LY; ++j) {
        int* e = &colv[(size_t)(64 + j) * 8];
        for (int b = 0; b < S; ++b) e[b] = cyv[(size_t)(j - 1) * S + b];
        const int64_t gy = (int64_t)(ny - cyv[(size_t)(j - 1) * S + gap]) * nx * pgap;
        accy += gy;
        e[6] = (int)gy;
        e[7] = (int)accy;
        maxstep = std::max(maxstep, gy);
      }
      for (int j = LY + 1; j < LY + 192; ++j) colv[(size_t)(64 + j) * 8 + 7] = (int)accy;  // (never traced)

      hcol.insert(hcol.end(), colv.begin(), colv.end());
      if ((int64_t)(LX + LY + 2) * maxstep + acc + accy >= (1ll << 30))
        return fail(NWK_EINVAL, "nwk_msa: profile DP of %d x %d columns would exceed int32", LX, LY);
      PairDesc& d = pd[q];
      memset(&d, 0, sizeof d);
      d.x_off = xoff;
      d.y_off = yoff;
      d.m = LX;
      d.n = LY;
      d.nbands = (int)ceil_div(LX, kProfBandRows);
      d.nchunks = (int)ceil_div(LY, 64);
      d.sblocks = d.nchunks + 1;
      d.slot = q;
      // the walk's diagonal-run fast path (trace_pair_affine<true>): merges of <= 16
      // sequences (k8 x 50k: 133 -> 140 e2e GCUPS; k64 / k256's wide profiles, whose
      // paths turn often, run slower with it)
      d.prio = nx + ny <= 16 ? 1 : 0;
      d.mat_off = mat;
      d.bnd_off = bnd;
      d.ops_off = ops;
      mat += (int64_t)d.nbands * prof_band_dwords(d.sblocks);
      bnd += (int64_t)d.nbands * d.nchunks * 64;  // granules of each band's last row (the last band's unused)
      ops += round_up((int64_t)LX + LY, 16);
      ntasks += d.nbands;
      st.cells += (double)LX * LY;
      st.matrix_bytes += 4 * (int64_t)d.nbands * prof_band_dwords(d.sblocks);
    }
    // ---- pack ints 0-5 of every profile entry for nw_profile<DOT> (rc_host / Prof::cnt keep the plain counts)
    // 5: every merge's columns are one sequence (a caterpillar guide tree's levels), so a
    // column's counts are one-hot and a cell's substitution cost is a byte select
    bool one_hot = true;
    for (int q = 0; q < np; ++q) one_hot = one_hot && prof[ms[q].y].members.size() == 1;
    int dot = maxpk < 256 ? (one_hot ? 5 : 4) : maxpk < 65536 ? 2 : 0;
    if (const char* ev = getenv("NWK_PROF_DOT")) {  // (A/B: caps the form)
      const int cap = atoi(ev);
      dot = std::min(dot, cap >= 5 ? 5 : cap >= 4 ? 4 : cap >= 2 ? 2 : 0);
      if (dot == 5 && !one_hot) dot = 4;
    }
    if (dot) {
      for (std::vector<int>* v : {&hrow, &hcol}) {
        for (size_t e = 0; e < v->size(); e += 8) {
          int* p = v->data() + e;
          if (dot == 5 && v == &hcol) {  // selector of the one symbol counted (none: bytes 0x0c = zero)
            uint32_t sel = 0x0c0c0c0cu;
            for (int b = 0; b < kProfSyms; ++b)
              if (p[b]) sel = 0x0c0c0c00u | (uint32_t)b;
            for (int b = 0; b < kProfSyms; ++b) p[b] = 0;
            p[0] = (int)sel;
            p[2] = p[6];
            continue;
          }
          uint32_t w[3] = {0, 0, 0};
          for (int b = 0; b < kProfSyms; ++b) {
            if (dot >= 4) w[b >> 2] |= (uint32_t)p[b] << (8 * (b & 3));
            else w[b >> 1] |= (uint32_t)p[b] << (16 * (b & 1));
          }
          for (int b = 0; b < kProfSyms; ++b) p[b] = b < 3 ? (int)w[b] : 0;
          p[dot >= 4 ? 2 : 3] = p[6];  // gy (gx) next to the counts: one 16-byte LDS read per column step
        }
      }
    }
    // ---- device buffers: [granules | matrices | ops | results]; the results (task
    // counter, err, and per merge done, endv = H(m, n), oplen, endij) follow the ops, so
    // a level zeroes them with one memset and reads them back with the ops in one copy
    t_build = now_ms();
    const int64_t bnd_b = round_up(bnd * 8 + 4096, 256), mat_b = round_up(mat * 4, 256), ops_b = round_up(ops, 256);
    const int64_t r_done = 256, r_endv = r_done + round_up(4 * (int64_t)np, 16), r_oplen = r_endv + round_up(4 * (int64_t)np, 16);
    const int64_t r_endij = r_oplen + round_up(4 * (int64_t)np, 16), res_b = round_up(r_endij + 8 * (int64_t)np, 256);
    const int64_t res_off = bnd_b + mat_b + ops_b;
    const int64_t work_b = res_off + res_b + 4096;
    if ((rc = d_mw.ensure((size_t)work_b)) != NWK_OK) return rc;
    if ((rc = d_prow.ensure(4 * hrow.size() + 64)) != NWK_OK) return rc;
    if ((rc = d_pcol.ensure(4 * hcol.size() + 64)) != NWK_OK) return rc;
    if ((rc = d_pd.ensure(sizeof(PairDesc) * np)) != NWK_OK) return rc;
    if ((rc = d_tk.ensure(sizeof(int2) * ntasks)) != NWK_OK) return rc;
    std::vector<int2> tk;
    for (int q = 0; q < np; ++q)
      for (int b = 0; b < pd[q].nbands; ++b) tk.push_back(make_int2(q, b));
    for (auto& d : pd) { d.mat_off += bnd_b / 4; d.ops_off += bnd_b + mat_b; }
    uint8_t* const res_d = d_mw.as<uint8_t>() + res_off;
    HIP_TRY(hipMemsetAsync(d_mw.p, 0, (size_t)bnd_b, c->stream));  // granule tags start below any epoch
    HIP_TRY(hipMemsetAsync(res_d, 0, (size_t)res_b, c->stream));
    HIP_TRY(hipMemcpyAsync(d_prow.p, hrow.data(), 4 * hrow.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_pcol.p, hcol.data(), 4 * hcol.size(), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_pd.p, pd.data(), sizeof(PairDesc) * np, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(d_tk.p, tk.data(), sizeof(int2) * ntasks, hipMemcpyHostToDevice, c->stream));
    FillArgs fa{};
    memset(&fa, 0, sizeof fa);
    fa.pairs = d_pd.as<PairDesc>();
    fa.tasks = d_tk.as<int2>();
    fa.ntasks = (int)ntasks;
    fa.mat = d_mw.as<uint32_t>();
    fa.bnd = d_mw.as<unsigned long long>();
    fa.counter = reinterpret_cast<unsigned*>(res_d);
    fa.err = reinterpret_cast<unsigned*>(res_d) + 16;
    fa.done = reinterpret_cast<unsigned*>(res_d + r_done);
    fa.ops = d_mw.as<uint8_t>();
    fa.oplen = reinterpret_cast<int*>(res_d + r_oplen);
    fa.endij = reinterpret_cast<int2*>(res_d + r_endij);
    fa.epoch = 1;
    fa.ntasks_pairs = np;
    fa.prow = d_prow.as<int>();
    fa.pcol = d_pcol.as<int>();
    fa.lin_mode = dot;  // the profile packing: nw_profile<5 | 4 | 2 | 0> (launch_fill)
    // fill-vs-walk guard: each merge's H(m, n) against the cost of its walked path (below)
    static const int msa_guard = getenv("NWK_GUARD") ? atoi(getenv("NWK_GUARD")) : 1;
    if (msa_guard != 0) fa.endv = reinterpret_cast<int*>(res_d + r_endv);
    const int grid = (int)std::min<int64_t>(fill_blocks_per_cu(kProfileDP, 4) * c->cus, ceil_div(ntasks, 4));
    if (getenv("NWK_WATCHDOG")) {
      if ((rc = c->d_prog.ensure(4 * (size_t)(grid + 1) * 4)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_prog.p, 0, 4 * (size_t)(grid + 1) * 4, c->stream));
      fa.prog = c->d_prog.as<unsigned>();
    }
    if (c->opts.verbose >= 3) {
      fprintf(stderr, "nwk_msa round %d: %d merges, %lld band tasks, grid %d\n", rd, np, (long long)ntasks, grid);
      fflush(stderr);
    }
    if (c->opts.verbose >= 2) {
      if ((rc = c->d_stamps.ensure(64 * (size_t)np)) != NWK_OK) return rc;
      HIP_TRY(hipMemsetAsync(c->d_stamps.p, 0, 64 * (size_t)np, c->stream));
      fa.stamps = c->d_stamps.as<unsigned long long>();
    }
    t_prep = now_ms();
    HIP_TRY(hipEventRecord(c->ev[0], c->stream));
    HIP_TRY(launch_fill(kProfileDP, 4, fa, grid, c->stream));
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    watchdog_wait(c, fa.prog, grid);
    // ops and results in one copy
    std::vector<uint8_t> hops((size_t)(ops_b + res_b));
    HIP_TRY(hipMemcpyAsync(hops.data(), d_mw.as<uint8_t>() + bnd_b + mat_b, hops.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint8_t* hres = hops.data() + ops_b;
    unsigned herr = 0;
    memcpy(&herr, hres + 64, 4);
    if (herr) return fail(NWK_EKERNEL, "nwk_msa: profile kernel fault (err=%u)", herr);
    std::vector<int> ol((size_t)np), mev((size_t)np, 0);
    std::vector<int2> ej((size_t)np);
    memcpy(ol.data(), hres + r_oplen, 4 * (size_t)np);
    memcpy(ej.data(), hres + r_endij, 8 * (size_t)np);
    if (fa.endv) memcpy(mev.data(), hres + r_endv, 4 * (size_t)np);
    t_wait = now_ms();
    float lvl_ms = 0;
    HIP_TRY(hipEventElapsedTime(&lvl_ms, c->ev[0], c->ev[1]));
    st.fill_ms += lvl_ms;
    ++st.fill_launches;
    ++st.batches;
    if (c->opts.verbose >= 2) {
      // per merge (8 u64): walk start / end (s_memrealtime, 100 MHz), then walk cycles
      // (s_memtime), of which tile switches and code reads, blocks << 32 | switches, moves
      std::vector<unsigned long long> sw((size_t)8 * np);
      HIP_TRY(hipMemcpy(sw.data(), fa.stamps, 64 * (size_t)np, hipMemcpyDeviceToHost));
      double wmax = 0, wsum = 0;
      int qm = 0;
      for (int q = 0; q < np; ++q) {
        const double w = sw[8 * q + 1] > sw[8 * q] ? (sw[8 * q + 1] - sw[8 * q]) * 1e-5 : 0.0;  // 100 MHz ticks -> ms
        if (w > wmax) wmax = w, qm = q;
        wsum += w;
      }
      const unsigned long long* x = &sw[8 * (size_t)qm];
      fprintf(stderr, "nwk_msa level %d: %d merges, %lld band tasks, %.3f ms (walks: longest %.3f ms, sum %.3f ms; "
              "longest: %llu cycles, tile switches %.1f%%, code reads %.1f%%, %llu blocks, %llu switches, %llu "
              "moves); host: previous merges + profiles %.3f ms (merges %.3f, profiles %.3f), uploads %.3f ms, launch "
              "to results %.3f ms\n", rd, np, (long long)ntasks, (double)lvl_ms, wmax, wsum, x[2], x[2] ? 100.0 * x[3] / x[2] : 0.0,
              x[2] ? 100.0 * x[4] / x[2] : 0.0, x[5] >> 32, x[5] & 0xffffffffull, x[6] & 0xffffffffull,
              t_build - t_lvl, t_mg - t_lvl, t_build - t_mg, t_prep - t_build, t_wait - t_prep);
    }
    // ---- merged profiles and merge costs (forward moves: prefix run, then the reversed trace)
    for (int q = 0; q < np; ++q) {
      const Prof &X = prof[ms[q].x], &Y = prof[ms[q].y];
      const int nx = (int)X.members.size(), ny = (int)Y.members.size();
      std::string mv;
      const int ei = ej[q].x, ejj = ej[q].y;
      if (ol[q] < 0 || ol[q] > X.len + Y.len || ei < 0 || ei > X.len || ejj < 0 || ejj > Y.len || (ei && ejj))
        return fail(NWK_EKERNEL, "nwk_msa: bad traceback (len %d, end %d,%d) for %d x %d", ol[q], ei, ejj, X.len, Y.len);
      mv.append((size_t)ei, 'U');
      mv.append((size_t)ejj, 'L');
      const uint8_t* o = hops.data() + (pd[q].ops_off - bnd_b - mat_b);
      for (int t = ol[q] - 1; t >= 0; --t) mv.push_back(o[t] == 'D' ? 'D' : (o[t] == 'u' || o[t] == 'U') ? 'U' : 'L');
      Prof& N = prof[ms[q].id];
      N.len = (int)mv.size();
      N.members = X.members;
      N.members.insert(N.members.end(), Y.members.begin(), Y.members.end());
      N.cnt.assign((size_t)N.len * S, 0);
      Prof &Xm = prof[ms[q].x], &Ym = prof[ms[q].y];
      Xm.up.assign((size_t)X.len, 0);
      Ym.up.assign((size_t)Y.len, 0);
      Xm.parent = Ym.parent = ms[q].id;
      int64_t cost = 0;
      int i = 0, j = 0;
      const std::vector<int>& rch = rc_host[q];
      const std::vector<int>& cyv = Y.cnt;
      for (int t = 0; t < N.len; ++t) {
        const char m = mv[(size_t)t];
        if ((m != 'L' && i >= X.len) || (m != 'U' && j >= Y.len))
          return fail(NWK_EKERNEL, "nwk_msa: traced path leaves the %d x %d matrix", X.len, Y.len);
        int* nc_t = &N.cnt[(size_t)t * S];
        if (m != 'L') {
          for (int b = 0; b < S; ++b) nc_t[b] += X.cnt[(size_t)i * S + b];
          Xm.up[(size_t)i] = t;
        } else {
          nc_t[gap] += nx;
        }
        if (m != 'U') {
          for (int b = 0; b < S; ++b) nc_t[b] += cyv[(size_t)j * S + b];
          Ym.up[(size_t)j] = t;
        } else {
          nc_t[gap] += ny;
        }
        if (m == 'D') {
          for (int b = 0; b < S; ++b) cost += (int64_t)rch[(size_t)i * 8 + b] * cyv[(size_t)j * S + b];
        } else if (m == 'U') {
          cost += rch[(size_t)i * 8 + 6];
        } else {
          cost += (int64_t)(ny - cyv[(size_t)j * S + gap]) * nx * pgap;
        }
        i += m != 'L';
        j += m != 'U';
      }
      if (i != X.len || j != Y.len) return fail(NWK_EKERNEL, "nwk_msa: traced path ends at (%d, %d) of (%d, %d)", i, j, X.len, Y.len);
      // the merge's walked path must cost the fill's H(m, n) (skel:274's ret = dp[m][n])
      if (fa.endv) {
        ++st.guard_checked;
        if (cost != (int64_t)mev[(size_t)q])
          return fail(NWK_EKERNEL, "nwk_msa: merge %d x %d: the walked path costs %lld but the fill's H(m, n) is %d",
                      X.len, Y.len, (long long)cost, mev[(size_t)q]);
      }
      *sop += cost;
      std::vector<int>().swap(Xm.cnt);
      std::vector<int>().swap(Ym.cnt);
    }
    t_lvl = t_wait;
    t_mg = now_ms();
  }
  st.total_ms = now_ms() - t_start;
  c->stats = st;
  if (c->opts.verbose)
    fprintf(stderr, "nwk_msa: k %d, %d levels, %.3g cells, fill %.3f ms (%.1f GCUPS), total %.3f ms\n", k, st.fill_launches,
            st.cells, st.fill_ms, st.fill_ms > 0 ? st.cells / st.fill_ms / 1e6 : 0.0, st.total_ms);
  const Prof& R = prof[nc - 1];
  if (R.len > cap) return fail(NWK_EINVAL, "nwk_msa: MSA length %d exceeds cap %lld", R.len, (long long)cap);
  *len = R.len;
  // rows, top down: a node's column -> MSA column (parents have larger ids than their children)
  std::vector<std::vector<int>> pos((size_t)nc);
  pos[nc - 1].resize((size_t)R.len);
  for (int t = 0; t < R.len; ++t) pos[nc - 1][(size_t)t] = t;
  for (int v = nc - 2; v >= 0; --v) {
    const Prof& P = prof[v];
    const std::vector<int>& pp = pos[(size_t)P.parent];
    pos[(size_t)v].resize((size_t)P.len);
    for (int t = 0; t < P.len; ++t) pos[(size_t)v][(size_t)t] = pp[(size_t)P.up[(size_t)t]];
    if (v >= k) continue;
    uint8_t* row = rows + (size_t)v * cap;
    memset(row, '_', (size_t)R.len);
    const uint8_t* sq = c->seqs.data() + c->off[v];
    for (int t = 0; t < P.len; ++t) row[pos[(size_t)v][(size_t)t]] = sq[t];
  }
  if (k == 1) memcpy(rows, c->seqs.data() + c->off[0], (size_t)R.len);
  return NWK_OK;
}

int nwk_get_minimum_penalties(const uint8_t* seqs, const int64_t* offsets, int32_t k, int32_t pxy, int32_t pgap,
                              int32_t* penalties, char* hash_hex, const nwk_opts* opts) {
  return min_penalties_sc(seqs, offsets, k, Scoring{pxy, pgap, false, 0, 0}, penalties, hash_hex, opts);
}

int nwk_get_minimum_penalties_affine(const uint8_t* seqs, const int64_t* offsets, int32_t k, int32_t pxy, int32_t go,
                                     int32_t ge, int32_t* penalties, char* hash_hex, const nwk_opts* opts) {
  return min_penalties_sc(seqs, offsets, k, Scoring{pxy, 0, true, go, ge}, penalties, hash_hex, opts);
}

}  // extern "C"
