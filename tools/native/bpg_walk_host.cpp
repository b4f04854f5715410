// Host build of the DEVICE one-lane BPG walks (bpg.h bpg_find_dev<W>, bpg_walk1) for bounds checking under
// AddressSanitizer (GPU ASan is not available): every program in its own exact-size allocation,
// the text padded as the engine pads it (ops/kernels.py padded_len), each (program, line) walked
// by bpg_find_dev<W> and by the host twin bpg_find_w<W>; prints the number of disagreements.
// Input files (tools/bpg_walk_check.py writes them): progs.bin = [count u64][len u64, words...]...,
// text.bin = padded bytes, lines.bin = [count u64][start i64, len i64]...
// Build: g++ -O1 -g -std=c++17 -fsanitize=address -I csrc/kernels tools/native/bpg_walk_host.cpp
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define __device__
#define __forceinline__ inline
#define __host__
#define __restrict__
#define LP_HD inline
#define __HIP__ 1
#define __ballot(x) ((unsigned long long)((x) ? 1 : 0))   // one lane: the wave is this lane
struct uint4 {
  uint32_t x, y, z, w;
};
inline uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
namespace lp {
inline int final_term_len(const uint8_t* s, int n) {
  if (n >= 1 && s[n - 1] == '\r') return 1;
  if (n >= 2 && s[n - 2] == 0xC2 && s[n - 1] == 0x85) return 2;
  if (n >= 3 && s[n - 3] == 0xE2 && s[n - 2] == 0x80 && (s[n - 1] == 0xA8 || s[n - 1] == 0xA9)) return 3;
  return 0;
}
}  // namespace lp
#include "bpg.h"

static std::vector<uint8_t> slurp(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) { std::perror(path); std::exit(2); }
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<uint8_t> v((size_t)n);
  if (n && std::fread(v.data(), 1, (size_t)n, f) != (size_t)n) std::exit(2);
  std::fclose(f);
  return v;
}

template <int W>
static bool dev_walk(const uint64_t* P, const uint8_t* s, int n) { return lp::bpg_find_dev<W>(P, s, n); }

static bool walk(const uint64_t* P, const uint8_t* s, int n) {
  switch ((int)(P[0] & 0xFF)) {
    case 1: return dev_walk<1>(P, s, n);
    case 2: return dev_walk<2>(P, s, n);
    case 3: return dev_walk<3>(P, s, n);
    case 4: return dev_walk<4>(P, s, n);
    case 6: return dev_walk<6>(P, s, n);
    default: return dev_walk<8>(P, s, n);
  }
}

int main(int argc, char** argv) {
  if (argc < 4) { std::fprintf(stderr, "usage: %s progs.bin text.bin lines.bin\n", argv[0]); return 2; }
  const std::vector<uint8_t> pb = slurp(argv[1]), tb = slurp(argv[2]), lb = slurp(argv[3]);
  const uint64_t* pw = reinterpret_cast<const uint64_t*>(pb.data());
  const uint64_t np = pw[0];
  std::vector<uint64_t*> progs;
  size_t o = 1;
  for (uint64_t i = 0; i < np; ++i) {
    const uint64_t len = pw[o++];
    uint64_t* p = static_cast<uint64_t*>(std::malloc(len * 8));   // exact size: ASan guards the end
    std::memcpy(p, pw + o, len * 8);
    o += len;
    progs.push_back(p);
  }
  uint8_t* text = static_cast<uint8_t*>(std::malloc(tb.size() + 0));
  std::memcpy(text, tb.data(), tb.size());
  // 16-byte alignment as on the device (hipMalloc); malloc under ASan aligns to 16 as well
  if (((uintptr_t)text & 15) != 0) { std::fprintf(stderr, "text not 16-byte aligned\n"); return 2; }
  const int64_t* lw = reinterpret_cast<const int64_t*>(lb.data());
  const int64_t nl = lw[0];
  long bad = 0, hits = 0, walks = 0;
  for (uint64_t i = 0; i < np; ++i) {
    const int W = (int)(progs[i][0] & 0xFF);
    if (W > lp::BPG_LANE_MAX_W) continue;
    for (int64_t x = 0; x < nl; ++x) {
      const uint8_t* s = text + lw[1 + 2 * x];
      const int n = (int)lw[2 + 2 * x];
      const bool d = walk(progs[i], s, n);
      const bool h = lp::bpg_find_host(progs[i], s, n);
      const bool l = W == 1 ? lp::bpg_walk1<const uint64_t*>(progs[i], s, n, true) : h;
      // the split walk (two parts OR'ed), as the device kernels run it on long lines
      bool sp = h;
      int mid = -1;
      if (W == 1 && n >= 32 && ((progs[i][0] >> 32) & 0xFFFFFFu) == 0) {
        for (int m = n / 2; m < n / 2 + 16 && m < n - 4; ++m)
          if (s[m - 1] < 0x80 && s[m] < 0x80) { mid = m; break; }
        if (mid > 0) {
          const int pk = lp::prev_of(lp::ascii_kind(s[mid - 1]));
          sp = lp::bpg_walk1<const uint64_t*>(progs[i], s, n, true, 0, mid) ||
               lp::bpg_walk1<const uint64_t*>(progs[i], s + mid, n - mid, true, pk);
        }
      }
      ++walks;
      hits += h;
      if (d != h || l != h || sp != h) {
        if (bad < 10)
          std::printf("mismatch prog %lu line %ld (n %d mid %d): dev %d lean %d split %d host %d\n", (unsigned long)i,
                      (long)x, n, mid, d, l, sp, h);
        ++bad;
      }
    }
  }
  std::printf("walks %ld hits %ld mismatches %ld\n", walks, hits, bad);
  for (auto* p : progs) std::free(p);
  std::free(text);
  return bad ? 1 : 0;
}
