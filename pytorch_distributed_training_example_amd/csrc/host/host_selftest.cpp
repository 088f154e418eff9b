// Host-side self-test of the extension's pure host logic, built with AddressSanitizer +
// UndefinedBehaviorSanitizer on the host half only (--cuda-host-only: no device code, no HIP
// runtime call is made, so it runs on a CPU-only machine). SURVEY.md §5 "race detection /
// sanitizers": the GPU half cannot be sanitized on this pool, the launch geometry and metadata
// packing that decide which memory every kernel touches can.
//
// Checked, for thousands of shapes each:
//   * multi_tensor.h mt_batches: every 16 Ki-element chunk of every tensor is covered by exactly one
//     workgroup, at most PDT_MT_MAX_TENSORS tensors per launch, chunk_start monotone;
//   * conv3x3_wgrad.hip geo_of / halo_rows: for every tile of an accepted shape the halo the kernel
//     stages fits the LDS buffer and the prefetch registers (brute force over all tiles), K rows fit,
//     the tiles cover every image row exactly once, and the splits cover every tile;
//   * conv3x3_wgrad.hip stride 2: the ResNet-50 block-0 shapes are accepted;
//   * conv1x1_wgrad.hip geo_of: the pixel splits cover every 32-pixel stage exactly once, the
//     workspace holds every split's partials, and the DMA source swizzle is a permutation of each
//     LDS row's chunks (every staged byte lands exactly once);
//   * batchnorm.hip reduce_geo3: the row blocks tile M exactly;
//   * embedding.hip workspace arithmetic.
// Build + run: python -m pytorch_distributed_training_example_amd._build --host-selftest
// (tests/test_host_asan.py does this on every CPU test run).
#include "../kernels/conv3x3_wgrad.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../multi_tensor.h"

namespace bn {
#include "../kernels/batchnorm.hip"
}
#include "../kernels/embedding.hip"
namespace w1 {
#include "../kernels/conv1x1_wgrad.hip"
}

static int g_fail = 0;
#define EXPECT(c, ...)                         \
  do {                                         \
    if (!(c)) {                                \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);                \
      std::printf("\n");                       \
      if (++g_fail > 20) std::exit(1);         \
    }                                          \
  } while (0)

static void test_mt_batches(std::mt19937_64& rng) {
  for (int trial = 0; trial < 2000; ++trial) {
    const int nt = 1 + (int)(rng() % 120);
    std::vector<int64_t> numel(nt);
    std::vector<void*> ptrs(nt);
    for (int t = 0; t < nt; ++t) {
      const int kind = (int)(rng() % 5);
      numel[t] = kind == 0 ? 0 : kind == 1 ? (int64_t)(rng() % 100) : kind == 2 ? PDT_MT_CHUNK * (int64_t)(rng() % 4)
                                                                    : (int64_t)(rng() % (64 << 20));
      ptrs[t] = reinterpret_cast<void*>((uintptr_t)(t + 1) << 20);
    }
    void* const* lists[1] = {ptrs.data()};
    std::vector<int64_t> covered(nt, 0);
    pdt::mt_batches<1>(nt, lists, numel.data(), [&](const MTMeta<1>& m, int nblocks) {
      EXPECT(m.ntensors >= 1 && m.ntensors <= PDT_MT_MAX_TENSORS, "ntensors %d", m.ntensors);
      EXPECT(m.chunk_start[0] == 0 && m.chunk_start[m.ntensors] == nblocks, "grid %d", nblocks);
      for (int k = 0; k < m.ntensors; ++k) {
        EXPECT(m.chunk_start[k + 1] > m.chunk_start[k], "empty tensor in a launch");
        const int t = (int)(((uintptr_t)m.ptr[0][k] >> 20) - 1);
        EXPECT(t >= 0 && t < nt && m.numel[k] == numel[t], "tensor identity");
        const int64_t nch = (m.numel[k] + PDT_MT_CHUNK - 1) / PDT_MT_CHUNK;
        EXPECT(m.chunk_start[k + 1] - m.chunk_start[k] == nch, "chunk count");
        covered[t] += nch;
      }
    });
    for (int t = 0; t < nt; ++t)
      EXPECT(covered[t] == (numel[t] + PDT_MT_CHUNK - 1) / PDT_MT_CHUNK, "tensor %d covered %lld", t,
             (long long)covered[t]);
  }
}

static void test_wgrad_geometry() {
  int accepted = 0;
  for (int H = 1; H <= 64; ++H)
    for (int W = 1; W <= 130; W += (W < 20 ? 1 : 7))
      for (int N : {1, 2, 3, 7, 64}) {
        for (int co : {64, 128}) {
          Geo g;
          if (!geo_of(N, H, W, 64, 256, co, 512, g)) continue;
          ++accepted;
          const int W2 = (W + 2 + 3) & ~3, H2 = H + 2;
          const int KP = (g.R * W + 15) & ~15;
          EXPECT(KP <= kp_max(1), "KP %d", KP);
          int64_t rows = 0;
          for (int t = 0; t < g.ntiles; ++t) {  // mirror of the kernel's load_tile
            const int g0 = t * g.R, gl = std::min(g0 + g.R, g.NH) - 1;
            const int prs = (g0 / H) * H2 + g0 % H, pre = (gl / H) * H2 + gl % H + 2;
            const int nh = (pre - prs + 1) * W2;
            EXPECT(nh <= halo_max(1), "N%d H%d W%d tile %d halo %d > %d", N, H, W, t, nh, halo_max(1));
            // the deepest B read (last pixel, tap 2,2) stays inside the staged rows
            const int gg = gl, w = W - 1;
            const int hr = ((gg / H) * H2 + gg % H - prs) * W2 + w + 2 * W2 + 2;
            EXPECT(hr < nh, "tap read row %d >= %d", hr, nh);
            rows += gl - g0 + 1;
          }
          EXPECT(rows == (int64_t)N * H, "tiles cover %lld of %d rows", (long long)rows, N * H);
          EXPECT((int64_t)g.nsplit * g.tiles_per_split >= g.ntiles && (g.nsplit - 1) * g.tiles_per_split < g.ntiles,
                 "splits");
          // exact prefetch tiling: the register pieces cover the LDS buffers exactly
          using C64 = WCfg<64, false>;
          using C128 = WCfg<128, true>;
          EXPECT(C64::kPfX * C64::kThreads == halo_max(1) * 8, "pfx");
          EXPECT(C128::kPfY * C128::kThreads == kp_max(1) * 16, "pfy");
        }
      }
  EXPECT(accepted > 1000, "only %d shapes accepted", accepted);
  // the ResNet-50 stride-1 3x3 shapes are all accepted at the bench batch
  for (int hw : {56, 28, 14, 7}) {
    Geo g;
    EXPECT(geo_of(1024, hw, hw, 64, 64, 64, 512, g), "ResNet-50 %dx%d rejected", hw, hw);
  }
}

static void test_wgrad1x1_geometry() {
  int accepted = 0;
  for (int M : {1, 31, 32, 33, 777, 4096, 50176, 200704, 3211264})
    for (int Ci : {64, 128, 192, 256, 512, 2048})
      for (int Co : {64, 128, 256, 320, 512, 2048}) {
        w1::W1Geo g;
        if (!w1::geo_of(M, Ci, Co, g)) continue;
        ++accepted;
        const w1::Blk blk = w1::pick_block(Co, Ci);
        const int kp = w1::info(blk, w1::variant_default(blk)).kp;
        EXPECT(g.ntiles * kp >= M && (g.ntiles - 1) * kp < M, "stages M=%d", M);
        if (g.ilv) {  // split k takes stages k, k + nsplit, ...: each stage exactly once
          int64_t covered = 0;
          for (int k = 0; k < g.nsplit; ++k) covered += (g.ntiles - k + g.nsplit - 1) / g.nsplit;
          EXPECT(g.nsplit <= g.ntiles && covered == g.ntiles, "interleaved stages M=%d", M);
        }
        EXPECT((int64_t)g.nsplit * g.tiles_per_split >= g.ntiles && (g.nsplit - 1) * g.tiles_per_split < g.ntiles,
               "splits M=%d Ci=%d Co=%d", M, Ci, Co);
        int cob, cib, occ;
        w1::block_dims(w1::pick_block(Co, Ci), cob, cib, occ);
        EXPECT(Co % cob == 0 && Ci % cib == 0 && g.nblk == (Co / cob) * (Ci / cib), "blocks Ci=%d Co=%d", Ci, Co);
        int ns = 0;
        EXPECT(w1::pdt_conv1x1_wgrad_ws_floats(M, Ci, Co, &ns) == (int64_t)ns * Ci * Co && ns == g.nsplit, "ws");
      }
  EXPECT(accepted > 300, "only %d 1x1 wgrad shapes accepted", accepted);
  for (int rowb : {128, 256, 512}) {
    for (int row = 0; row < 32; ++row) {
      std::vector<int> seen(rowb / 16, 0);
      for (int slot = 0; slot < rowb / 16; ++slot) {
        const int ch = rowb == 128 ? w1::swz<128>(row, slot) : (rowb == 256 ? w1::swz<256>(row, slot) : w1::swz<512>(row, slot));
        EXPECT(ch >= 0 && ch < rowb / 16, "swizzle range");
        if (ch >= 0 && ch < rowb / 16) ++seen[ch];
      }
      for (int c = 0; c < rowb / 16; ++c) EXPECT(seen[c] == 1, "swizzle not a permutation rowb %d row %d", rowb, row);
    }
  }
}

static void test_bn_geometry() {
  for (int64_t M : {1LL, 7LL, 49LL, 1000LL, 25088LL, 3211264LL})
    for (int C : {64, 128, 256, 512, 1024, 2048})
      for (int U : {2, 4, 8}) {
        const bn::ReduceGeo g = bn::reduce_geo3(M, C, U);
        EXPECT(g.nrow >= 1 && (int64_t)g.nrow * g.rows_per_block >= M && (int64_t)(g.nrow - 1) * g.rows_per_block < M,
               "bn rows M=%lld C=%d", (long long)M, C);
      }
}

int main() {
  std::mt19937_64 rng(12345);
  test_mt_batches(rng);
  test_wgrad_geometry();
  test_bn_geometry();
  test_wgrad1x1_geometry();
  for (int hw : {56, 28, 14}) {
    Geo g;
    EXPECT(geo_of(1024, (hw - 1) / 2 + 1, (hw - 1) / 2 + 1, 2 * 64, 2 * 64, 128, 256, g, 2, hw, hw),
           "ResNet-50 stride-2 %dx%d rejected", hw, hw);
  }
  EXPECT(pdt_embedding_bwd_ws_ints(8192, 50304) == 3 * 50304 + 2 * 8192, "embedding ws");
  std::printf(g_fail ? "host selftest: %d failures\n" : "host selftest: all passed (%d)\n", g_fail);
  return g_fail ? 1 : 0;
}
