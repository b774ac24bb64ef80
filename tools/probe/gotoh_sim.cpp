// gotoh_sim.cpp -- host run of gotoh_bits.h's step, one cell per call (bit 0
// of every plane), to check the bit-sliced algebra exactly.
//
// stdin:  pxy go ge [trace]
//         then one pair per line: x y   (any bytes but whitespace)
// stdout: H[m][n] per pair (the affine score, oracle nwo_score_affine); with
//         `trace`, "H a1 a2" per pair: the walk of nwo_pair_affine over the
//         step's four stored bits (D, Fsrc, Eext, Fext) and the prefix trim
//
// Built by tests/test_gotoh_bits_probe.py (g++ -O2), which compares its output
// with the oracle on random pairs.
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

#include "../../multiple-sequence-alignment-openmp-openmpi_amd/csrc/nwk_gotoh_planes.h"

using namespace gotoh_bits;

template <class C>
static long long score(const std::string& x, const std::string& y, int go, int ge, std::vector<uint8_t>* tb) {
  const int m = (int)x.size(), n = (int)y.size();
  if (m == 0 || n == 0) return (m + n) == 0 ? 0 : go + (long long)(m + n) * ge;
  if (tb) tb->assign((size_t)(m + 1) * (n + 1), 0);
  constexpr int NQ1 = C::NQ > 0 ? C::NQ : 1;
  struct Down { uint32_t h[C::NV], f[NQ1]; };
  std::vector<Down> up(n + 1);  // row i-1's h and f per column
  for (int j = 1; j <= n; ++j) {  // row 0: h(0, j) = G(0, j-1) - G(0, j), F' = +inf
    const_v<C>(j == 1 ? -go : 0, up[j].h);
    const_q<C>(go, up[j].f);
  }
  long long sum_h = 0;
  for (int i = 1; i <= m; ++i) {
    uint32_t L[C::NV], eL[NQ1];
    const_v<C>(i == 1 ? -go : 0, L);  // v(i, 0) = G(i-1, 0) - G(i, 0); E'(i, 0) = +inf
    const_q<C>(go, eL);
    for (int j = 1; j <= n; ++j) {
      const uint32_t match = x[i - 1] == y[j - 1] ? ~0u : 0u;
      uint32_t v[C::NV], e[NQ1], h[C::NV], f[NQ1], D, Fs, Ee, Fe;
      step<C>(match, L, eL, up[j].h, up[j].f, v, e, h, f, D, Fs, Ee, Fe);
      if (tb) (*tb)[(size_t)i * (n + 1) + j] = (uint8_t)((D & 1u) | (Fs & 1u) << 1 | (Ee & 1u) << 2 | (Fe & 1u) << 3);
      for (int p = 0; p < C::NV; ++p) {
        L[p] = v[p];
        up[j].h[p] = h[p];
      }
      for (int q = 0; q < NQ1; ++q) {
        eL[q] = e[q];
        up[j].f[q] = f[q];
      }
      if (i == m) {
        int hv = C::VLO;
        for (int p = 0; p < C::NV; ++p) hv += (int)(h[p] & 1u);
        sum_h += hv;
      }
    }
  }
  // G(m, n) = G(m, 0) - sum_j h(m, j), G(m, 0) = go; H = G + (m + n) ge
  return go - sum_h + (long long)(m + n) * ge;
}

// nwo_pair_affine's walk (oracle/nw_oracle.c:240-270) over the stored bits
static void walk(const std::string& x, const std::string& y, const std::vector<uint8_t>& tb, std::string& a1,
                 std::string& a2) {
  const int m = (int)x.size(), n = (int)y.size(), l = m + n;
  std::string xa(l + 1, ' '), ya(l + 1, ' ');
  int i = m, j = n, xp = l, yp = l, st = 0;  // 0 H, 1 F, 2 E
  while (!(i == 0 || j == 0)) {
    const uint8_t b = tb[(size_t)i * (n + 1) + j];
    if (st == 0) {
      if (b & 1u) { xa[xp--] = x[i - 1]; ya[yp--] = y[j - 1]; --i; --j; continue; }
      st = (b & 2u) ? 1 : 2;
    }
    if (st == 1) { st = (b & 8u) ? 1 : 0; xa[xp--] = x[i - 1]; ya[yp--] = '_'; --i; }
    else { st = (b & 4u) ? 2 : 0; xa[xp--] = '_'; ya[yp--] = y[j - 1]; --j; }
  }
  while (xp > 0) xa[xp--] = i > 0 ? x[--i] : '_';
  while (yp > 0) ya[yp--] = j > 0 ? y[--j] : '_';
  int id = 1;
  for (int a = l; a >= 1; --a)
    if (ya[a] == '_' && xa[a] == '_') { id = a + 1; break; }
  a1 = xa.substr(id);
  a2 = ya.substr(id);
}

static bool g_trace = false;

template <int GO, int GE, int PXY>
static bool run_if(int pxy, int go, int ge, const std::vector<std::pair<std::string, std::string>>& prs) {
  if (pxy != PXY || go != GO || ge != GE) return false;
  for (auto& p : prs) {
    std::vector<uint8_t> tb;
    const long long H = score<Cfg<GO, GE, PXY>>(p.first, p.second, go, ge, g_trace ? &tb : nullptr);
    if (!g_trace) { std::printf("%lld\n", H); continue; }
    std::string a1, a2;
    walk(p.first, p.second, tb, a1, a2);
    std::printf("%lld %s %s\n", H, a1.empty() ? "-" : a1.c_str(), a2.empty() ? "-" : a2.c_str());
  }
  return true;
}

int main() {
  int pxy, go, ge;
  std::string first;
  if (!std::getline(std::cin, first) || std::sscanf(first.c_str(), "%d %d %d", &pxy, &go, &ge) != 3) return 2;
  g_trace = first.find("trace") != std::string::npos;
  std::vector<std::pair<std::string, std::string>> prs;
  std::string x, y;
  while (std::cin >> x >> y) prs.emplace_back(x, y);
  // the instantiated scorings (C5's 3/3/1 first)
  if (run_if<3, 1, 3>(pxy, go, ge, prs) || run_if<0, 2, 3>(pxy, go, ge, prs) || run_if<2, 1, 1>(pxy, go, ge, prs) ||
      run_if<5, 2, 4>(pxy, go, ge, prs) || run_if<1, 1, 0>(pxy, go, ge, prs))
    return 0;
  std::fprintf(stderr, "gotoh_sim: scoring %d/%d/%d not instantiated\n", pxy, go, ge);
  return 3;
}
