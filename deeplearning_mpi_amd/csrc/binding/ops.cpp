// Torch binding of the gfx950 kernel library: tensor plumbing, conv geometry planning (forward,
// sub-pixel data-gradient phases, transposed conv, split-K weight-gradient) and tile selection.
// Every function launches on the current HIP stream and never synchronises, so a whole training
// step can be captured into a hipGraph.
#include "ops.h"

#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <string>
#include <vector>
#include <stdexcept>

#include "../kernels/dlmpi_kernels.h"

namespace dlmpi_ext {

using dlmpi::ConvArgs;
using dlmpi::ConvPhase;
using dlmpi::FinArgs;
using dlmpi::Stream1x1Args;
using dlmpi::DgradStreamArgs;
using dlmpi::make_fastdiv;
using dlmpi::WgradArgs;

static inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

static inline void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("dlmpi kernel launch failed: ") + what + ": " +
                                                hipGetErrorString(e));
}

template <typename T>
static inline T* ptr(const at::Tensor& t) {
  return reinterpret_cast<T*>(t.data_ptr());
}
template <typename T>
static inline T* optr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

static inline void require_gpu(const at::Tensor& t, const char* name) {
  if (!t.is_cuda()) throw std::runtime_error(std::string(name) + " must be a GPU tensor");
}

static inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Activation storage type: bf16 (the product path) or fp32 (the fp32 precision path).  Every
// activation operand of one launch must share it; the kernels are instantiated for both.
static inline int act_f32(const at::Tensor& t, const char* what) {
  if (t.scalar_type() == at::kFloat) return 1;
  if (t.scalar_type() == at::kBFloat16) return 0;
  throw std::runtime_error(std::string(what) + ": activations must be bf16 or fp32");
}
static inline void same_type(const at::Tensor& ref, const c10::optional<at::Tensor>& t, const char* what) {
  if (t.has_value() && t->defined() && t->scalar_type() != ref.scalar_type())
    throw std::runtime_error(std::string(what) + ": operand dtype differs from the activations'");
}
static inline void same_type(const at::Tensor& ref, const at::Tensor& t, const char* what) {
  same_type(ref, c10::optional<at::Tensor>(t), what);
}

// K-iteration constants: the reduction step (64 bf16 / 32 fp32 elements = one 128-byte LDS row)
// walks channels (C a multiple of it) or, for small C, every 16-byte piece is its own tap
static void set_kstep(ConvArgs& a, int C) {
  if (C % 8 != 0) throw std::runtime_error("conv: channel count must be a multiple of 8 (pad it)");
  if (a.f32) {   // conv_igemm.hip launch_f32: C < 32 or C % 32 != 0 -> small-channel staging
    a.cstep = C % 32 == 0 ? 32 : 0;
    a.tstep = 0;
    return;
  }
  if (C >= 64) {
    if (C % 64 != 0) throw std::runtime_error("conv: channels >= 64 must be a multiple of 64");
    a.cstep = 64;
    a.tstep = 0;
  } else {
    if (64 % C != 0) throw std::runtime_error("conv: channels < 64 must divide 64");
    a.cstep = 0;
    a.tstep = 64 / C;
  }
}

// Tile choice.  256x128 (per-wave 128x64: 25 % less LDS traffic per MFMA than 128x128) wins on
// long reductions into wide outputs (UNet 3x3 convs with >= 256 channels: up to 1.3x, measured by
// benchmarks/conv_bench.py) and loses on the short / memory-bound ResNet GEMMs; 64-row tiles for
// small grids.  `red` = GEMM reduction length (R*S*C).
constexpr int kBm256MinTiles = 256;

// Shortest 1x1 reduction (red == cin) that takes the 256-row tile
// (default 1024: the 14^2 1024->256 forward and 256<-1024 data gradient, 128x128 -> 256x128 tiles
// halve the B-operand re-reads, -14 % each; ResNet-50 +0.8 %, profiles/r3_bm256red); other
// reductions from 2304 as before
constexpr int kBm256MinRed1x1 = 1024;

// cin: channel count of the GEMM's gathered operand
static void pick_tiles(int64_t M, int Kout, int64_t red, int cin, int& bm, int& bn, bool pro = false,
                       bool wide1x1 = true) {
  bn = Kout <= 64 ? 64 : 128;
  // 64 (mod 128) channels above 128 (the UNet's 192-channel top concat gradient): 64-wide tiles
  // cover them exactly instead of a half-empty last 128-wide tile (a third more MFMA work)
  if (Kout > 128 && Kout % 128 == 64) bn = 64;
  bm = 128;
  const int64_t nt = (Kout + bn - 1) / bn;
  const int64_t tiles = ((M + 127) / 128) * nt;
  // 64-channel outputs: 256 x 64 tiles (4 x 1 waves of 64 x 64).  Measured (conv_bench): wins for
  // the small-channel stems (-13 % ResNet 7x7, -10 % UNet first conv) and the 4M-row UNet level-1
  // 3x3s (-4 %), loses 3-8 % on the 0.8M-row ResNet layer1 GEMMs -> only there.
  if (bn == 64 && (M + 255) / 256 >= 512 && (cin < 64 || (M >= (2 << 20) && red >= 576))) bm = 256;
  else if (Kout >= 256 && (red >= 2304 || (wide1x1 && red == cin && red >= kBm256MinRed1x1)) && ((M + 255) / 256) * nt >= kBm256MinTiles) bm = 256;
  else if (tiles < 512) bm = 64;
  // grids that do not fill the chip even with 64-row tiles (ResNet-18 on 32 x 32 CIFAR: 8-128 tiles):
  // 64-wide output tiles too -- twice the blocks before split-K (the autotuner's choice on every such
  // layer, forward and data gradient: +5 % CIFAR img/s, profiles/r4_cifar).  Not for fused BN-apply
  // consumers (pro): their one output column is what lets column 0 alone store the applied input;
  // two columns would each recompute the prologue (profiles/r3_fuse_apply_2col_rejected).
  if (!pro && bm == 64 && bn == 128 && ((M + 63) / 64) * nt < 256) bn = 64;
}

// ---- pipelined 8-wave tiles (conv_igemm.hip conv_pipe_kernel) -----------------------------------
// Long reductions over >= 64-channel operands into 256-multiple outputs: one 8-wave block per CU
// with an LDS ring instead of 2-3 single-stage 4-wave blocks.  Of the pipelined tiles (256 x 256,
// 224 x 256, 128 x 256) the one with the least modeled time: rounds of the 256-CU chip x tile area
// x a per-area cost (128 x 256: per-wave 64 x 64 tiles, 1.25x the LDS traffic per MFMA of the
// 128 x 64 per-wave tiles of the others; profiles/r4_lab).  At batch 256 the 14^2 ResNet layers are
// 50,176 rows: 196 tiles of 256 rows leave 60 CUs idle, 224 tiles of 224 rows 32.  Returns the kernel
// variant + 1 (0: keep the single-stage tile bm x bn).  g_pipe_override (tests): -1 the rule, 0 never,
// 1 wherever the kernel applies.
static int g_pipe_override = -1;
static int g_pipe_dgrad_override = -1;   // dlmpi_ext set_conv_pipe_dgrad (A/B): 0 keeps data gradients off it
// conv_igemm.hip VAR of the DMA issue: A pieces before the first K-half of MFMAs, B pieces before the
// second (2) for the 256 / 224-row tiles; additionally staggered over the two waves of a SIMD (4) for
// 128 x 256 (profiles/r4_lab: 3-8 % over issuing all at once, on every measured shape)
static int pipe_select(int f32, int pro, int cin, int64_t M, int Kout, int64_t red, int& bm, int& bn) {
  if (f32 || pro != 0 || cin % 64 != 0 || cin > 4032 || g_pipe_override == 0) return 0;   // (conv_igemm.hip kPipeMaxC)
  if (g_pipe_override == 1) {
    bm = Kout >= 256 ? 256 : (Kout > 64 ? 256 : 512);
    bn = Kout >= 256 ? 256 : (Kout > 64 ? 128 : 64);
    return 2 + 1;
  }
  if (Kout < 256 || Kout % 256 != 0 || red < 1024) return 0;
  struct Cand { int bm; double unit; };
  const Cand cands[] = {{256, 1.0}, {224, 1.0}, {128, 1.25}};
  double best = 1e300;
  int pbm = 256;
  for (const Cand& c : cands) {
    const int64_t tiles = ((M + c.bm - 1) / c.bm) * (Kout / 256);
    const double t = (double)((tiles + 255) / 256) * c.bm * c.unit;
    if (t < best - 1e-9) {
      best = t;
      pbm = c.bm;
    }
  }
  // one block per CU and no split-K: small grids (ResNet-18 on 32 x 32 CIFAR reaches 2 tiles) stay
  // on the single-stage kernel, which splits their K over otherwise idle CUs
  if (((M + pbm - 1) / pbm) * (Kout / 256) < 96) return 0;
  bm = pbm;
  bn = 256;
  return (bm == 128 ? 4 : 2) + 1;
}

// ---- the producer's BN-apply fused into a 1x1 consumer (conv_igemm.hip conv1x1_apply_kernel) ----
// pro-3 launches whose Kout is one 64 / 128 / 256-channel tile column run the register-staged kernel
// (128-row tiles: 64-row tiles measured slower, profiles/r5_apply) instead of the single-stage pro-3
// conv_igemm_kernel.  set_conv_apply(0): the latter.  Every other pro-3 launch -- and one whose
// operands the register-staged kernel cannot address (apply_launch_ok) -- runs the single-stage kernel
// on 128 x 64 tiles (kPro3Bm x kPro3Bn; the larger pro-3 tiles spilled and are not built), so both
// paths produce ceil(M / 128) BN-statistics rows and the caller's buffer fits either.
static int g_apply_override = -1;
constexpr int kPro3Bm = 128, kPro3Bn = 64;
static bool apply_kernel(int f32, int pro, int C, int K, int R, int S, int stride, int pad) {
  return g_apply_override != 0 && pro == 3 && !f32 && R == 1 && S == 1 && stride == 1 && pad == 0 &&
         dlmpi_conv1x1_apply_ok(C, K);
}
// the launch-time conditions of dlmpi_conv1x1_apply beyond the shape: 16-byte output rows and 32-bit
// element offsets of every operand
static bool apply_launch_ok(const ConvArgs& a) {
  const int64_t ld = std::max<int64_t>(a.ldx, std::max<int64_t>(a.ldpz, a.ldpy));
  return a.vec_store && (int64_t)a.Nimg * a.H * a.W * ld < (1ll << 31);
}

// ---- 2-D halo tiles for 3x3 / stride-1 / pad-1 convolutions (conv_igemm.hip HALO) ----------------
// set_conv_halo(0) (tests): these convolutions through the im2col gather path too.
static int g_halo_override = -1;   // dlmpi_ext set_conv_halo (tests)
static int g_splitk_override = 0;   // dlmpi_ext set_conv_splitk (tests): > 0 forces that many K slices
static bool halo_on() { return g_halo_override != 0; }
// Tile th x tw (th * tw <= bm, (th + 2) * (tw + 2) <= 192 / 352 rows for bm 128 / 256) covering a
// P x Q grid with the fewest tiles (ties: the wider tile).
static void halo_geom(int P, int Q, int bm, int& th, int& tw, int& tiles_h, int& tiles_w) {
  int best = INT32_MAX;
  const int rows = bm == 256 ? 352 : 192;   // conv_igemm.hip HALO_ROWS
  for (int w = bm == 256 ? 32 : 16; w >= 4; --w) {
    const int h = std::min(bm / w, rows / (w + 2) - 2);
    if (h < 1) continue;
    const int t = ceil_div(P, h) * ceil_div(Q, w);
    if (t < best) {
      best = t;
      th = h;
      tw = w;
    }
  }
  tiles_h = ceil_div(P, th);
  tiles_w = ceil_div(Q, tw);
}
// Halo tile shape (profiles/r4_halo): 256-pixel tiles (16 x 16, 18 x 18 halo) for 64-channel
// outputs (+9 % on 56^2 / 512^2 grids: half the B-fragment reads per MFMA) and for >= 256-channel
// outputs (+2-4 %); 128-pixel tiles for 128-channel outputs, where the 256 x 128 tile loses 4-7 %.
static void halo_tiles(int Kout, int& bm, int& bn) {
  bn = std::min(bn, 128);
  bm = (bn == 64 || Kout >= 256) ? 256 : 128;
}
// Measured per shape (profiles/r3_halo): halo tiles win 1-6 % on grids >= 28 x 28 against the
// 128-row gather tiles, tie with the 8-wave 256 x 256 tiles, and lose on 14^2 / 7^2 grids (a
// 7 x 7 image fills a 126-pixel tile to 39 %) -- so only there, and not instead of 256 x 256 tiles.
static bool halo_eligible(int f32, int pro, int C, int R, int S, int stride, int pad, int P, int Q) {
  if (!halo_on() || f32 || pro != 0 || C % 64 != 0 || R != 3 || S != 3 || stride != 1 || pad != 1) return false;
  return g_halo_override == 2 || (P >= 28 && Q >= 28);   // 2: any grid (tests)
}
// Halo tiles before the pipelined kernel for >= 256 output channels (profiles/r4_halo: the 256 x 128
// halo tile beat the best pipe tile on every UNet 3x3 of >= 32^2 grid, 2-5 %; 32^2 1024 -> 1024: 231.6
// vs 243.2 us); the pipe kernel keeps the 14^2 / 7^2 grids, where halo tiles are not eligible.
static int g_halo_first = 1;   // dlmpi_ext set_halo_first (A/B): 0 = the pipelined kernel first where it applies
static bool halo_first(bool halo_ok, int Kout) { return halo_ok && Kout >= 256 && g_halo_first; }
static int g_halo_ran = 0;   // 1 if the last conv2d_fwd / conv2d_dgrad ran halo tiles (tests)
// Switch a fully set-up single-phase launch (bm 128 / 256) to halo tiles: its M-tiles (and stats rows)
// become N x tiles_h x tiles_w.
static void apply_halo(ConvArgs& a, int N, int bm) {
  ConvPhase& p = a.ph[0];
  int th = 8, tw = 16, tiles_h = 1, tiles_w = 1;
  halo_geom(p.P, p.Q, bm, th, tw, tiles_h, tiles_w);
  a.halo = 1;
  a.th = th;
  a.tw = tw;
  a.tiles_h = tiles_h;
  a.tiles_w = tiles_w;
  a.fd_tw = make_fastdiv((uint32_t)tw);
  a.fd_tilesw = make_fastdiv((uint32_t)tiles_w);
  a.fd_thw = make_fastdiv((uint32_t)(tiles_h * tiles_w));
  p.mtiles = N * tiles_h * tiles_w;
  p.tile_base = 0;
}
static int halo_mtiles(int N, int P, int Q, int Kout, int bn) {
  int th = 8, tw = 16, tiles_h = 1, tiles_w = 1, bm = 128;
  halo_tiles(Kout, bm, bn);
  halo_geom(P, Q, bm, th, tw, tiles_h, tiles_w);
  return N * tiles_h * tiles_w;
}

// ---- conv tile autotuner ("benchmark mode", the reference's cudnn.benchmark = True,
// /root/reference/pytorch/resnet/main.py:29) --------------------------------------------------------
// At batch 256 most ResNet-50 layers quantize badly on 256 CUs (784 tiles of a 14^2 layer on 768
// resident-block slots take two tile-times).  The first time a (conv, pass, epilogue) signature is
// launched outside a hipGraph capture, every valid (BM, BN, split-K) plan is timed on the real
// operands with the device otherwise idle and the fastest is cached for the process; later calls
// (and captures) use the cached plan.  Outputs are overwritten by every trial (the epilogues are
// idempotent; BN partials go to a scratch buffer), so the call's result is the chosen plan's.
// DLMPI_CONV_AUTOTUNE=1 turns it on; default 0 = the static tile rules only (run-to-run
// bit-reproducible plans): ResNet-50 measured +0.3 %, inside the noise (12,407 / 12,458 img/s on vs
// 12,385 / 12,397 off, profiles/r3_autotune), while timing-chosen plans make two processes of the
// same job sum in different orders.
struct ConvPlan {
  int bm, bn, splitk_req;
};
static std::map<std::string, ConvPlan> g_conv_plans;
static int g_autotune_override = -1;
static bool conv_autotune_on() {
  static const int v = [] {
    const char* e = getenv("DLMPI_CONV_AUTOTUNE");
    return e ? atoi(e) : 0;   // 2: also log every plan to stderr
  }();
  return (g_autotune_override >= 0 ? g_autotune_override : v) != 0;
}

static std::string conv_key(const ConvArgs& a, int pass) {
  std::string k = std::to_string(pass);
  auto add = [&](int64_t v) { k += ',' + std::to_string(v); };
  add(a.f32); add(a.Nimg); add(a.H); add(a.W); add(a.C); add(a.ldx); add(a.Kout); add(a.ldw); add(a.S);
  add(a.OH); add(a.OW); add(a.ldy); add(a.so); add(a.sa); add(a.nphase); add(a.kvalid); add(a.vec_store);
  add(a.out_f32); add(a.bias != nullptr); add(a.res != nullptr); add(a.scale != nullptr); add(a.relu);
  add(a.stats != nullptr); add(a.nstat); add(a.mask != nullptr); add(a.mscale != nullptr); add(a.mbits != nullptr);
  add(a.z != nullptr); add(a.z2 != nullptr); add(a.pro);
  for (int i = 0; i < a.nphase; ++i) {
    const ConvPhase& p = a.ph[i];
    add(p.P); add(p.Q); add(p.Tr); add(p.Ts); add(p.dh0); add(p.dw0); add(p.wr0); add(p.ws0);
  }
  return k;
}

// (re)tile a fully set-up launch for BM x BN: M-tiles and stats bases of every phase
static int apply_tiles(ConvArgs& a, int bm, int bn) {
  a.ntiles = ceil_div(a.Kout, bn);
  int t = 0;
  for (int i = 0; i < a.nphase; ++i) {
    ConvPhase& p = a.ph[i];
    p.mtiles = ceil_div((int64_t)a.Nimg * p.P * p.Q, bm);
    p.tile_base = t;
    t += p.mtiles;
  }
  return t;
}

// Plan for a fully set-up (default-tiled) launch: the cached one, or tune now.  Returns false if
// autotuning does not apply (the caller keeps its static plan).
static bool conv_plan(ConvArgs& a, int pass, int& bm, int& bn) {
  if (!conv_autotune_on() || a.pro != 0 || a.halo) return false;
  // trials re-run the launch: an output that is also one of its inputs (in-place residual / mask /
  // z) would be transformed once per trial -- keep the static plan there
  const void* y = a.y;
  if (y == a.x || y == a.res || y == a.z || y == a.z2 || y == a.mask) return false;
  const std::string key = conv_key(a, pass);
  auto it = g_conv_plans.find(key);
  if (it == g_conv_plans.end()) {
    hipStream_t st = cur_stream();
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return false;
    int maxk = 0;
    for (int i = 0; i < a.nphase; ++i) maxk = std::max(maxk, a.ph[i].ksteps);
    std::vector<ConvPlan> cands;
    const int tiles_m[] = {64, 128, 256};
    for (int tbm : tiles_m)
      for (int tbn : {64, 128, 256}) {
        if (tbn > 64 && a.Kout <= tbn / 2) continue;   // mostly padding
        if (tbm == 256 && tbn == 256 && a.C < 64) continue;
        if (tbm == 128 && tbn == 256 && a.C < 64) continue;
        if (tbm == 64 && tbn == 256) continue;
        if (a.f32 && (tbm > 128 || tbn > 128)) continue;   // launch_f32's tiles
        cands.push_back({tbm, tbn, 0});
        if (maxk >= 16) cands.push_back({tbm, tbn, 2});
        if (maxk >= 8) cands.push_back({tbm, tbn, 1});
      }
    // BN partials of the trials: scratch rows for the smallest tile
    at::Tensor scratch;
    float* real_stats = a.stats;
    if (a.stats) {
      ConvArgs t = a;
      const int rows = apply_tiles(t, 64, 64);
      scratch = at::empty({(int64_t)rows * a.nstat * a.Kout}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA));
    }
    check(hipDeviceSynchronize(), "autotune sync");
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    ConvPlan best{bm, bn, 0};
    float best_ms = 1e30f;
    for (const ConvPlan& c : cands) {
      ConvArgs t = a;
      apply_tiles(t, c.bm, c.bn);
      t.splitk_req = c.splitk_req;
      if (t.stats) t.stats = ptr<float>(scratch);
      if (dlmpi_conv_igemm(&t, c.bm, c.bn, st) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      hipEventRecord(e0, st);
      for (int r = 0; r < 3; ++r) (void)dlmpi_conv_igemm(&t, c.bm, c.bn, st);
      hipEventRecord(e1, st);
      if (hipEventSynchronize(e1) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best_ms) {
        best_ms = ms;
        best = c;
      }
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    a.stats = real_stats;
    if (getenv("DLMPI_CONV_AUTOTUNE") && atoi(getenv("DLMPI_CONV_AUTOTUNE")) == 2)
      fprintf(stderr, "[dlmpi autotune] pass %d %s -> %dx%d split %d (%.1f us; static %dx%d)\n", pass, key.c_str(),
              best.bm, best.bn, best.splitk_req, best_ms / 3 * 1000, bm, bn);
    it = g_conv_plans.emplace(key, best).first;
  }
  bm = it->second.bm;
  bn = it->second.bn;
  a.splitk_req = it->second.splitk_req;
  apply_tiles(a, bm, bn);
  return true;
}

// fp32: single-stage 4-wave tiles only, at most 128 x 128 (launch_f32)
static void f32_tiles(int& bm, int& bn) {
  bm = std::min(bm, 128);
  bn = std::min(bn, 128);
}

static void finish_phase(ConvPhase& p, int Nimg, int C, int bm, bool f32 = false) {
  p.mtiles = ceil_div((int64_t)Nimg * p.P * p.Q, bm);
  p.ksteps = ceil_div((int64_t)p.Tr * p.Ts * C, f32 ? 32 : 64);
  if (p.Tr * p.Ts == 0) p.ksteps = 0;
  p.fdPQ = make_fastdiv((uint32_t)std::max(1, p.P * p.Q));
  p.fdQ = make_fastdiv((uint32_t)std::max(1, p.Q));
  p.fdTs = make_fastdiv((uint32_t)std::max(1, p.Ts));
}

static void fill_epilogue(ConvArgs& a, at::Tensor& y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
                          const c10::optional<at::Tensor>& res, int ldres, int resoff,
                          const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& shift, bool relu,
                          const c10::optional<at::Tensor>& stats) {
  a.y = y.data_ptr();
  a.out_f32 = y.scalar_type() == at::kFloat ? 1 : 0;
  a.ldy = ldy;
  a.yoff = yoff;
  a.kvalid = a.Kout;
  a.bias = optr<float>(bias);
  a.res = optr<uint16_t>(res);
  a.ldres = ldres;
  a.resoff = resoff;
  a.scale = optr<float>(scale);
  a.shift = optr<float>(shift);
  a.relu = relu ? 1 : 0;
  a.stats = optr<float>(stats);
  a.nstat = 2;
}

// Extras of a pro-3 launch (conv2d_fwd_bn_apply sets them around the shared forward path).
struct Pro3Extra {
  const float* rscale;
  const float* rshift;
  uint16_t* y;
  int ldy, yoff;
  uint8_t* mbits;
};
static thread_local const Pro3Extra* g_pro3 = nullptr;

// Operand prologue of the gathered operand (ConvArgs::pro 3): (k0 scale, k1 shift, pz = residual) of
// the producer block's BN-apply + residual + ReLU, computed and stored by the consumer's prologue.
static void set_prologue(ConvArgs& a, int pro, const c10::optional<at::Tensor>& k0, const c10::optional<at::Tensor>& k1,
                         const c10::optional<at::Tensor>& pz, int ldpz, int pzoff) {
  a.pro = pro;
  if (pro == 0) return;
  if (pro != 3) throw std::runtime_error("conv prologue: mode 3 (the producer's pending BN-apply) or none");
  if (a.C < 64 || a.C % 64) throw std::runtime_error("conv prologue: channel count must be a multiple of 64");
  a.pscale = optr<float>(k0);
  a.pshift = optr<float>(k1);
  a.pz = optr<uint16_t>(pz);
  a.ldpz = ldpz;
  a.pzoff = pzoff;
  const Pro3Extra* e = g_pro3;
  if (!e || !a.pscale || !a.pshift || !a.pz || !e->y || !e->mbits || k0->numel() < a.C || k1->numel() < a.C ||
      (ldpz | pzoff | e->ldy | e->yoff) % 8 || ((e->rscale != nullptr) != (e->rshift != nullptr)) || a.f32)
    throw std::runtime_error("conv prologue 3: scale / shift, an aligned residual, y and mask bits required");
  a.prscale = e->rscale;
  a.prshift = e->rshift;
  a.py = e->y;
  a.ldpy = e->ldy;
  a.pyoff = e->yoff;
  a.pmbits = e->mbits;
}

static at::Tensor colsum_ws(const at::Tensor& like, int T, int C);

// The streaming 1x1 kernel (conv1x1_stream.hip) applies to this forward conv: its statistics have
// one row per block of an N-tile (G rows) instead of one per M-tile.  Shape-only decision (the
// stats buffer is sized from it before the launch); the launch checks the rest (alignment, sizes).
static int g_stream_ran = 0;   // 1 if the last conv2d_fwd ran the streaming 1x1 kernel (tests)
static int g_dgrad_stream_ran = 0;   // 1 if the last conv2d_dgrad ran the streaming 1x1 kernel (tests)

static bool stream1x1_shape(int64_t M, int C, int K, int R, int S, int stride, int pad, int pro, int f32, int& bm,
                            int& bn, int& G) {
  if (R != 1 || S != 1 || (stride != 1 && stride != 2) || pad != 0 || pro != 0 || f32) return false;
  return dlmpi_stream1x1_plan(M, C, K, stride, &bm, &bn, &G) != 0;
}

// The streaming 3x3 kernel (conv3x3_stream.hip: 64 -> 64 channels, stride 1, pad 1) applies: shape-only
// decision, as stream1x1_shape (its statistics have G rows, one per block).  Its grid shares the
// RCCL-aware budget of the streaming data gradient (one block per CU).
static int g_conv3_ran = 0;   // 1 if the last conv2d_fwd / conv2d_dgrad ran the streaming 3x3 kernel (tests)
static int g_head_ran = 0;           // 1 if the last conv2d_fwd ran the 1x1 head kernel (head.hip)
static int g_head_on = 1;            // dlmpi_ext set_head1x1 (A/B)
static int g_c8_ran = 0;             // 1 if the last conv2d_fwd ran the 8-channel 3x3 kernel (conv_small.hip)
static int g_c8_on = 1;              // dlmpi_ext set_conv_c8 (A/B)
static int g_convT_stream = 1;       // dlmpi_ext set_convT_stream (A/B)
static int g_convT_stream_ran = 0;   // 1 if the last convT2x2_fwd ran the streaming kernel

// 3x3 / s1 / p1 from an 8-channel (padded image) input into 64 channels: conv_small.hip
static bool c8_shape(int64_t M, int C, int K, int R, int S, int stride, int pad, int W, int pro, int f32, int& G) {
  if (!g_c8_on || C != 8 || K != 64 || R != 3 || S != 3 || stride != 1 || pad != 1 || W % 16 || pro || f32)
    return false;
  G = dlmpi_conv3x3_c8_blocks(M);
  return true;
}
// the ResNet stem on its 2x2 space-to-depth image (4x4 / s1 / p0, 16 channels -> 64): conv_small.hip
static int g_c16_on = 1;    // dlmpi_ext set_conv_c16 (A/B)
static int g_c16_ran = 0;   // 1 if the last conv2d_fwd ran it
static bool c16_shape(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int pro, int f32, int& G) {
  if (!g_c16_on || C != 16 || K != 64 || R != 4 || S != 4 || stride != 1 || pad != 0 || H < 4 || (W - 3) % 16 ||
      W < 19 || pro || f32)
    return false;
  G = dlmpi_conv4x4_c16_blocks((int64_t)N * (H - 3) * (W - 3));
  return true;
}
static bool stream3x3_shape(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int pro, int f32,
                            int& th, int& tw, int& G) {
  if (R != 3 || S != 3 || stride != 1 || pad != 1 || pro != 0 || f32) return false;
  return dlmpi_conv3_stream_plan(N, H, W, C, K, dlmpi_dgs_blocks(), &th, &tw, &G) != 0;
}
static dlmpi::Conv3StreamArgs conv3_args(const at::Tensor& x, int N, int H, int W, int ldx, int xoff, const at::Tensor& w,
                                         int flip, void* y, int ldy, int yoff, int th, int tw, int G) {
  dlmpi::Conv3StreamArgs c{};
  c.x = ptr<uint16_t>(x);
  c.ldx = ldx; c.xoff = xoff;
  c.w = ptr<uint16_t>(w);
  c.ldw = 9 * 64; c.flip = flip;
  c.y = reinterpret_cast<uint16_t*>(y);
  c.ldy = ldy; c.yoff = yoff;
  c.N = N; c.H = H; c.W = W;
  c.th = th; c.tw = tw;
  c.tiles_h = ceil_div(H, th);
  c.tiles_w = ceil_div(W, tw);
  c.ntiles = N * c.tiles_h * c.tiles_w;
  c.G = G;
  return c;
}



// y[n, p, q, yoff + k] = epilogue( sum_{r,s,c} x[n, p*stride - pad + r, q*stride - pad + s, xoff + c] * w[k][r][s][c] )
// fin (with stats): also finalize the BatchNorm over these statistics -- inside the launch when the
// in-launch finalize is available, else by the standalone finalize right after it.
static int conv2d_fwd_impl(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K, int R,
               int S, int stride, int pad, at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
               const c10::optional<at::Tensor>& res, int ldres, int resoff, const c10::optional<at::Tensor>& scale,
               const c10::optional<at::Tensor>& shift, bool relu, const c10::optional<at::Tensor>& stats, int bm_req,
               int kvalid, int bn_req, int pro, const c10::optional<at::Tensor>& pk0,
               const c10::optional<at::Tensor>& pk1, const c10::optional<at::Tensor>& pz, int ldpz, int pzoff,
               const FinArgs* fin);

int conv2d_fwd_pro(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K, int R,
               int S, int stride, int pad, at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
               const c10::optional<at::Tensor>& res, int ldres, int resoff, const c10::optional<at::Tensor>& scale,
               const c10::optional<at::Tensor>& shift, bool relu, const c10::optional<at::Tensor>& stats, int bm_req,
               int kvalid, int bn_req, int pro, const c10::optional<at::Tensor>& pk0,
               const c10::optional<at::Tensor>& pk1, const c10::optional<at::Tensor>& pz, int ldpz, int pzoff) {
  return conv2d_fwd_impl(x, N, H, W, C, ldx, xoff, w, K, R, S, stride, pad, y, ldy, yoff, bias, res, ldres, resoff,
                         scale, shift, relu, stats, bm_req, kvalid, bn_req, pro, pk0, pk1, pz, ldpz, pzoff, nullptr);
}

// conv2d_fwd_pro + the training BatchNorm finalize of its statistics (scale / shift / saved mean and
// invstd / running statistics), as one launch when possible.
int conv2d_fwd_bn(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K, int R,
                  int S, int stride, int pad, at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
                  const at::Tensor& stats, int pro, const c10::optional<at::Tensor>& pk0,
                  const c10::optional<at::Tensor>& pk1, const c10::optional<at::Tensor>& pz, int ldpz, int pzoff,
                  double count, const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                  const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
                  double momentum, double eps, at::Tensor bnscale, at::Tensor bnshift,
                  const c10::optional<at::Tensor>& save_mean, const c10::optional<at::Tensor>& save_invstd) {
  FinArgs f{};
  f.mode = 0;
  f.count = count;
  f.gamma = optr<float>(gamma);
  f.beta = optr<float>(beta);
  f.running_mean = optr<float>(running_mean);
  f.running_var = optr<float>(running_var);
  f.momentum = (float)momentum;
  f.eps = (float)eps;
  f.scale = ptr<float>(bnscale);
  f.shift = ptr<float>(bnshift);
  f.save_mean = optr<float>(save_mean);
  f.save_invstd = optr<float>(save_invstd);
  return conv2d_fwd_impl(x, N, H, W, C, ldx, xoff, w, K, R, S, stride, pad, y, ldy, yoff, bias, c10::nullopt, 0, 0,
                         c10::nullopt, c10::nullopt, false, stats, 0, 0, 0, pro, pk0, pk1, pz, ldpz, pzoff, &f);
}

// conv2d_fwd_bn whose input is the PRODUCER's pending BN-apply: x = that BN's input z (scale, shift),
// res = its residual (rscale / rshift: a BN-output residual applied on the fly); the conv's operand
// prologue (pro 3) computes relu(z * scale + shift + res), consumes it AND stores it to yapp with
// its ReLU mask bits -- the standalone BN-apply pass and the consumer's re-read of its output go.
int conv2d_fwd_bn_apply(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K,
                        at::Tensor z, int ldz, int zoff, const c10::optional<at::Tensor>& bias, const at::Tensor& stats,
                        const at::Tensor& ascale, const at::Tensor& ashift, const at::Tensor& res, int ldres,
                        int resoff, const c10::optional<at::Tensor>& rscale, const c10::optional<at::Tensor>& rshift,
                        at::Tensor yapp, int ldyapp, int yappoff, at::Tensor mbits, double count,
                        const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                        const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
                        double momentum, double eps, at::Tensor bnscale, at::Tensor bnshift,
                        const c10::optional<at::Tensor>& save_mean, const c10::optional<at::Tensor>& save_invstd) {
  same_type(x, res, "conv2d_fwd_bn_apply res");
  same_type(x, yapp, "conv2d_fwd_bn_apply y");
  if (mbits.scalar_type() != at::kByte || mbits.numel() < (int64_t)N * H * W * (C / 8))
    throw std::runtime_error("conv2d_fwd_bn_apply: mask bits [pixels][C/8] uint8 required");
  Pro3Extra e{optr<float>(rscale), optr<float>(rshift), ptr<uint16_t>(yapp), ldyapp, yappoff, ptr<uint8_t>(mbits)};
  g_pro3 = &e;
  try {
    const int r = conv2d_fwd_bn(x, N, H, W, C, ldx, xoff, w, K, 1, 1, 1, 0, z, ldz, zoff, bias, stats, 3, ascale,
                                ashift, res, ldres, resoff, count, gamma, beta, running_mean, running_var, momentum,
                                eps, bnscale, bnshift, save_mean, save_invstd);
    g_pro3 = nullptr;
    return r;
  } catch (...) {
    g_pro3 = nullptr;
    throw;
  }
}

static void run_fin_after(const at::Tensor& stats, int rows, int K, const FinArgs* fin);
static int g_c3pro_on = 1;   // dlmpi_ext set_conv3_pro (A/B): 0 = the standalone BN-apply before the conv
// The streaming 64 -> 64 3x3 forward takes this launch with the producer's BN-apply + ReLU fused
// (conv3x3_stream_kernel PRO): shape and operand conditions (the model asks before it defers the apply).
static bool conv3_pro_ok(int N, int H, int W, int C, int K, int ldx, int xoff, int ldz, int zoff, int ldyapp,
                         int yappoff) {
  int th, tw, G;
  return g_c3pro_on && C == 64 && K == 64 && stream3x3_shape(N, H, W, C, K, 3, 3, 1, 1, 0, 0, th, tw, G) &&
         ldx % 8 == 0 && xoff % 8 == 0 && ldz % 8 == 0 && zoff % 8 == 0 && ldyapp % 8 == 0 && yappoff % 8 == 0 &&
         (int64_t)H * W * std::max(ldz, ldyapp) * 2 < (1ll << 31);
}
// conv2d_fwd_bn of a 3x3 / s1 / p1 64 -> 64 conv whose input is the producer's pending BN-apply + ReLU
// (no residual): x = that BN's input z, (ascale, ashift) its coefficients; the streaming kernel applies
// them to its staged halo and stores the applied input to yapp (each pixel once).  Returns the
// statistics rows (G), or -1 if the fused launch does not apply (the caller applies first).
int conv3x3_fwd_bn_apply(const at::Tensor& x, int N, int H, int W, int ldx, int xoff, const at::Tensor& w,
                         at::Tensor z, int ldz, int zoff, const c10::optional<at::Tensor>& bias, const at::Tensor& stats,
                         const at::Tensor& ascale, const at::Tensor& ashift, at::Tensor yapp, int ldyapp, int yappoff,
                         double count, const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                         const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
                         double momentum, double eps, at::Tensor bnscale, at::Tensor bnshift,
                         const c10::optional<at::Tensor>& save_mean, const c10::optional<at::Tensor>& save_invstd) {
  require_gpu(x, "conv3x3_fwd_bn_apply x");
  if (act_f32(x, "conv3x3_fwd_bn_apply") || z.scalar_type() != at::kBFloat16 || yapp.scalar_type() != at::kBFloat16 ||
      !conv3_pro_ok(N, H, W, 64, 64, ldx, xoff, ldz, zoff, ldyapp, yappoff) || ascale.numel() < 64 ||
      ashift.numel() < 64)
    return -1;
  int th, tw, G;
  stream3x3_shape(N, H, W, 64, 64, 3, 3, 1, 1, 0, 0, th, tw, G);
  if (stats.size(0) < G) throw std::runtime_error("conv3x3_fwd_bn_apply: stats buffer too small");
  dlmpi::Conv3StreamArgs c = conv3_args(x, N, H, W, ldx, xoff, w, 0, z.data_ptr(), ldz, zoff, th, tw, G);
  c.bias = optr<float>(bias);
  c.stats = ptr<float>(stats);
  c.psc = ptr<float>(ascale);
  c.psh = ptr<float>(ashift);
  c.py = ptr<uint16_t>(yapp);
  c.ldpy = ldyapp;
  c.pyoff = yappoff;
  check(dlmpi_conv3x3_stream(&c, 0, cur_stream()), "conv3x3_fwd_bn_apply");
  g_conv3_ran = 1;
  FinArgs f{};
  f.mode = 0;
  f.count = count;
  f.gamma = optr<float>(gamma);
  f.beta = optr<float>(beta);
  f.running_mean = optr<float>(running_mean);
  f.running_var = optr<float>(running_var);
  f.momentum = (float)momentum;
  f.eps = (float)eps;
  f.scale = ptr<float>(bnscale);
  f.shift = ptr<float>(bnshift);
  f.save_mean = optr<float>(save_mean);
  f.save_invstd = optr<float>(save_invstd);
  run_fin_after(stats, G, 64, &f);
  return G;
}

// the BN finalize of a forward conv's statistics [rows][2][K]
static void run_fin_after(const at::Tensor& stats, int rows, int K, const FinArgs* fin) {
  at::Tensor ws = colsum_ws(stats, rows, K);
  check(dlmpi_bn_finalize(ptr<float>(stats), rows, K, fin->count, fin->gamma, fin->beta, fin->running_mean,
                          fin->running_var, fin->momentum, fin->eps, fin->scale, fin->shift, fin->save_mean,
                          fin->save_invstd, ptr<double>(ws), cur_stream()),
        "bn_finalize");
}

static int conv2d_fwd_impl(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K, int R,
               int S, int stride, int pad, at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
               const c10::optional<at::Tensor>& res, int ldres, int resoff, const c10::optional<at::Tensor>& scale,
               const c10::optional<at::Tensor>& shift, bool relu, const c10::optional<at::Tensor>& stats, int bm_req,
               int kvalid, int bn_req, int pro, const c10::optional<at::Tensor>& pk0,
               const c10::optional<at::Tensor>& pk1, const c10::optional<at::Tensor>& pz, int ldpz, int pzoff,
               const FinArgs* fin) {
  require_gpu(x, "x");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  ConvArgs a{};
  a.f32 = act_f32(x, "conv2d_fwd");
  same_type(x, w, "conv2d_fwd w");
  same_type(x, res, "conv2d_fwd res");
  a.x = ptr<uint16_t>(x);
  a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.xoff = xoff;
  a.w = ptr<uint16_t>(w);
  a.ldw = R * S * C;
  a.S = S;
  a.OH = P; a.OW = Q;
  a.so = 1; a.sa = stride;
  a.Nimg = N; a.Kout = K;
  fill_epilogue(a, y, ldy, yoff, bias, res, ldres, resoff, scale, shift, relu, stats);
  if (kvalid > 0 && kvalid < K) a.kvalid = kvalid;
  a.vec_store = (a.kvalid == a.Kout && (ldy % 8) == 0 && (yoff % 8) == 0) ? 1 : 0;
  set_kstep(a, C);
  set_prologue(a, pro, pk0, pk1, pz, ldpz, pzoff);
  int bm, bn;
  pick_tiles((int64_t)N * P * Q, K, (int64_t)R * S * C, C, bm, bn, pro != 0);
  if (a.f32) f32_tiles(bm, bn);
  const bool halo_ok = bm_req <= 0 && bn_req <= 0 && halo_eligible(a.f32, pro, C, R, S, stride, pad, P, Q);
  int pipe = bm_req <= 0 && bn_req <= 0 && !halo_first(halo_ok, K)
                 ? pipe_select(a.f32, pro, C, (int64_t)N * P * Q, K, (int64_t)R * S * C, bm, bn) : 0;
  const bool halo = !pipe && halo_ok;
  if (halo) halo_tiles(K, bm, bn);
  if (bm_req > 0) bm = bm_req;   // tests / experiments: force a tile shape
  if (bn_req > 0) bn = bn_req;
  if (bn_req == 256) {   // 256-column tiles (128 x 256, 256 x 256) exist only as the pipelined 8-wave kernel
    if (a.f32 || pro != 0 || C % 64 != 0 || (bm != 128 && bm != 256))
      throw std::runtime_error("conv2d_fwd: 256-column tiles need bf16, no prologue, C % 64 == 0, 128 / 256 rows");
    pipe = (bm == 128 ? 4 : 2) + 1;
  }
  g_stream_ran = 0;
  g_conv3_ran = 0;
  g_head_ran = 0;
  g_c8_ran = 0;
  {  // the UNet input conv: 8-channel image -> 64, 3x3
    int G;
    if (bm_req <= 0 && bn_req <= 0 && c8_shape((int64_t)N * H * W, C, K, R, S, stride, pad, W, pro, a.f32, G)) {
      const bool ok = !res.has_value() && !scale.has_value() && !relu && a.kvalid == K && ldx % 8 == 0 &&
                      xoff % 8 == 0 && ldy % 8 == 0 && yoff % 8 == 0 && (int64_t)N * H * W < (1ll << 31) &&
                      y.scalar_type() == at::kBFloat16;
      if (ok) {
        if (a.stats && stats->size(0) < G) throw std::runtime_error("conv2d_fwd: stats buffer too small");
        check(dlmpi_conv3x3_c8(a.x, ldx, xoff, N, H, W, a.w, a.bias, a.y, ldy, yoff, a.stats, G, cur_stream()),
              "conv2d_fwd (8-channel 3x3)");
        g_c8_ran = 1;
        if (fin != nullptr) run_fin_after(*stats, G, K, fin);
        return G;
      }
    }
  }
  g_c16_ran = 0;
  {  // the ResNet stem (space-to-depth image, 16 channels -> 64, 4x4 taps)
    int G;
    if (bm_req <= 0 && bn_req <= 0 && c16_shape(N, H, W, C, K, R, S, stride, pad, pro, a.f32, G)) {
      const bool ok = !res.has_value() && !scale.has_value() && !relu && a.kvalid == K && ldx % 8 == 0 &&
                      xoff % 8 == 0 && ldy % 8 == 0 && yoff % 8 == 0 && (int64_t)N * H * W * ldx < (1ll << 31) &&
                      (int64_t)N * P * Q * ldy < (1ll << 31) && y.scalar_type() == at::kBFloat16 && a.ldw == 256;
      if (ok) {
        if (a.stats && stats->size(0) < G) throw std::runtime_error("conv2d_fwd: stats buffer too small");
        check(dlmpi_conv4x4_c16(a.x, ldx, xoff, N, H, W, a.w, a.bias, a.y, ldy, yoff, a.stats, G, cur_stream()),
              "conv2d_fwd (stem 4x4 x 16 channels)");
        g_c16_ran = 1;
        if (fin != nullptr) run_fin_after(*stats, G, K, fin);
        return G;
      }
    }
  }
  {  // <= 4 output channels, 1x1, no epilogue beyond the bias (the UNet head): a streaming dot product
    const int kv = a.kvalid > 0 ? a.kvalid : K;
    if (g_head_on && bm_req <= 0 && bn_req <= 0 && pro == 0 && !a.f32 && R == 1 && S == 1 && stride == 1 &&
        pad == 0 && !stats.has_value() && !res.has_value() && !scale.has_value() && !relu && fin == nullptr &&
        dlmpi_head1x1_ok(C, kv) && ldx % 8 == 0 && xoff % 8 == 0 &&
        (y.scalar_type() == at::kFloat || y.scalar_type() == at::kBFloat16)) {
      check(dlmpi_head1x1(a.x, ldx, xoff, (int64_t)N * H * W, C, a.w, a.ldw, a.bias, a.y, ldy, yoff, kv,
                          y.scalar_type() == at::kFloat ? 1 : 0, nullptr, nullptr, cur_stream()),
            "conv2d_fwd (1x1 head)");
      g_head_ran = 1;
      return 0;
    }
  }
  {  // streaming 3x3 kernel (64 -> 64: the full-resolution UNet layers, ResNet layer-1 conv2)
    int th, tw, G;
    if (bm_req <= 0 && bn_req <= 0 && stream3x3_shape(N, H, W, C, K, R, S, stride, pad, pro, a.f32, th, tw, G)) {
      const bool ok = !res.has_value() && !scale.has_value() && !relu && a.kvalid == K && a.vec_store &&
                      ldx % 8 == 0 && xoff % 8 == 0 && (int64_t)H * W * ldy * 2 < (1ll << 31) &&
                      y.scalar_type() == at::kBFloat16 && w.scalar_type() == at::kBFloat16;
      if (ok) {
        if (a.stats && stats->size(0) < G) throw std::runtime_error("conv2d_fwd: stats buffer too small");
        dlmpi::Conv3StreamArgs c = conv3_args(x, N, H, W, ldx, xoff, w, 0, a.y, ldy, yoff, th, tw, G);
        c.bias = a.bias;
        c.stats = a.stats;
        check(dlmpi_conv3x3_stream(&c, a.stats ? 0 : 1, cur_stream()), "conv2d_fwd (stream 3x3)");
        g_conv3_ran = 1;
        if (fin != nullptr) {
          at::Tensor ws = colsum_ws(*stats, G, K);
          check(dlmpi_bn_finalize(a.stats, G, K, fin->count, fin->gamma, fin->beta, fin->running_mean,
                                  fin->running_var, fin->momentum, fin->eps, fin->scale, fin->shift, fin->save_mean,
                                  fin->save_invstd, ptr<double>(ws), cur_stream()),
                "bn_finalize");
        }
        return G;
      }
    }
  }
  {  // streaming 1x1 kernel (short reductions into wide, memory-bound outputs)
    const int64_t M = (int64_t)N * P * Q;
    int sbm, sbn, G;
    if (bm_req <= 0 && bn_req <= 0 && stream1x1_shape(M, C, K, R, S, stride, pad, pro, a.f32, sbm, sbn, G)) {
      const bool ok = !res.has_value() && !scale.has_value() && !relu && a.kvalid == K && a.vec_store &&
                      ldx % 8 == 0 && xoff % 8 == 0 && (int64_t)N * H * W * ldx < (1ll << 31) &&
                      M * ldy * 2 < (1ll << 31) && y.scalar_type() == at::kBFloat16;
      if (ok) {
        Stream1x1Args sa{};
        sa.x = ptr<uint16_t>(x);
        sa.ldx = ldx; sa.xoff = xoff;
        sa.w = ptr<uint16_t>(w);
        sa.y = reinterpret_cast<uint16_t*>(a.y);
        sa.ldy = ldy; sa.yoff = yoff;
        sa.y_bytes = (int)std::min<int64_t>(INT32_MAX, (int64_t)y.numel() * 2);
        sa.M = (int)M; sa.C = C; sa.Kout = K;
        sa.bias = a.bias;
        sa.stats = a.stats;
        sa.G = G; sa.ntiles = K / sbn; sa.mtiles = ceil_div(M, sbm);
        sa.s2 = stride == 2 ? 1 : 0;
        sa.H = H; sa.W = W;
        sa.fdPQ = make_fastdiv((uint32_t)(P * Q));
        sa.fdQ = make_fastdiv((uint32_t)Q);
        if (a.stats && stats->size(0) < G) throw std::runtime_error("conv2d_fwd: stats buffer too small");
        check(dlmpi_conv1x1_stream(&sa, sbm, sbn, cur_stream()), "conv2d_fwd (stream 1x1)");
        g_stream_ran = 1;
        if (fin != nullptr) {
          at::Tensor ws = colsum_ws(*stats, G, K);
          check(dlmpi_bn_finalize(a.stats, G, K, fin->count, fin->gamma, fin->beta, fin->running_mean,
                                  fin->running_var, fin->momentum, fin->eps, fin->scale, fin->shift, fin->save_mean,
                                  fin->save_invstd, ptr<double>(ws), cur_stream()),
                "bn_finalize");
        }
        return G;
      }
    }
  }
  if (pro == 3 && (R != 1 || S != 1 || stride != 1 || pad != 0))
    throw std::runtime_error("conv prologue 3: a 1x1 / stride-1 conv");
  const bool fused_apply = bm_req <= 0 && bn_req <= 0 && apply_kernel(a.f32, pro, C, K, R, S, stride, pad) &&
                           apply_launch_ok(a);
  if (fused_apply) {
    bm = kPro3Bm;
    bn = K;
  } else if (pro == 3) {
    bm = kPro3Bm;
    bn = kPro3Bn;
  }
  a.ntiles = ceil_div(K, bn);
  a.nphase = 1;
  ConvPhase& p = a.ph[0];
  p.P = P; p.Q = Q; p.Tr = R; p.Ts = S;
  p.dh0 = -pad; p.dhs = 1; p.dw0 = -pad; p.dws = 1;
  p.wr0 = 0; p.wrs = 1; p.ws0 = 0; p.wss = 1;
  p.oh0 = 0; p.ow0 = 0;
  finish_phase(p, N, C, bm, a.f32);
  if (fused_apply) {
    if (fin != nullptr && (!a.stats || stats->size(0) < p.mtiles))
      throw std::runtime_error("conv2d_fwd_bn: stats [mtiles][2][K] required");
    check(dlmpi_conv1x1_apply(&a, bm, cur_stream()), "conv2d_fwd (fused apply 1x1)");
    if (fin != nullptr) run_fin_after(*stats, p.mtiles, K, fin);
    return p.mtiles;
  }
  if (halo) apply_halo(a, N, bm);
  g_halo_ran = halo ? 1 : 0;
  // autotuned tiling: BN-stats launches only through conv2d_fwd_bn (its buffer is sized for the
  // largest row count, conv2d_fwd_mtiles_pro, and its finalize uses the actual one)
  if (!pipe && (fin != nullptr || !a.stats) && bm_req <= 0 && bn_req <= 0) conv_plan(a, 0, bm, bn);
  if (fin != nullptr && (!a.stats || stats->size(0) < p.mtiles))
    throw std::runtime_error("conv2d_fwd_bn: stats [mtiles][2][K] required");
  if (g_splitk_override > 0) a.splitk_req = g_splitk_override;
  check(dlmpi_conv_igemm_ex(&a, bm, bn, pipe, cur_stream()), "conv2d_fwd");
  if (fin != nullptr) {   // the BN finalize of these statistics
    at::Tensor ws = colsum_ws(*stats, p.mtiles, K);
    check(dlmpi_bn_finalize(a.stats, p.mtiles, K, fin->count, fin->gamma, fin->beta, fin->running_mean,
                            fin->running_var, fin->momentum, fin->eps, fin->scale, fin->shift, fin->save_mean,
                            fin->save_invstd, ptr<double>(ws), cur_stream()),
          "bn_finalize");
  }
  return p.mtiles;   // rows of the stats partial buffer
}

// The 1x1 head (<= 4 outputs) over a deferred BN-apply + ReLU input relu(z * scale + shift) (the UNet's
// last decoder BN output, never stored): head.hip with the apply computed on the fly.
void conv1x1_head_affine(const at::Tensor& z, int N, int H, int W, int C, int ldz, int zoff, const at::Tensor& w,
                         int ldw, int kv, const at::Tensor& scale, const at::Tensor& shift, at::Tensor y, int ldy,
                         int yoff, const c10::optional<at::Tensor>& bias) {
  require_gpu(z, "z");
  if (act_f32(z, "conv1x1_head_affine") || !dlmpi_head1x1_ok(C, kv) || ldz % 8 || zoff % 8 ||
      scale.numel() < C || shift.numel() < C || (y.scalar_type() != at::kFloat && y.scalar_type() != at::kBFloat16))
    throw std::runtime_error("conv1x1_head_affine: bf16 z, C in 16..512, <= 4 outputs, aligned rows");
  check(dlmpi_head1x1(z.data_ptr(), ldz, zoff, (int64_t)N * H * W, C, w.data_ptr(), ldw, optr<float>(bias),
                      y.data_ptr(), ldy, yoff, kv, y.scalar_type() == at::kFloat ? 1 : 0, ptr<float>(scale),
                      ptr<float>(shift), cur_stream()),
        "conv1x1_head_affine");
  g_head_ran = 1;
}

int conv2d_fwd(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w, int K, int R,
               int S, int stride, int pad, at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias,
               const c10::optional<at::Tensor>& res, int ldres, int resoff, const c10::optional<at::Tensor>& scale,
               const c10::optional<at::Tensor>& shift, bool relu, const c10::optional<at::Tensor>& stats, int bm_req,
               int kvalid, int bn_req) {
  return conv2d_fwd_pro(x, N, H, W, C, ldx, xoff, w, K, R, S, stride, pad, y, ldy, yoff, bias, res, ldres, resoff,
                        scale, shift, relu, stats, bm_req, kvalid, bn_req, 0, c10::nullopt, c10::nullopt,
                        c10::nullopt, 0, 0);
}

// Forward conv whose output is the gradient of y = relu(BN(z)) (a BN+ReLU without residual): the
// epilogue applies the ReLU mask [z * mscale + mshift > 0] before the store and emits that BN's
// backward partials [tiles][2][K] = {sum v, sum v*z}, returned.  (UNet: the ConvTranspose2d
// data-gradient -- a 2x2/s2 conv -- into the DoubleConv output below it.)
at::Tensor conv2d_fwd_bnbwd(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, const at::Tensor& w,
                            int K, int R, int S, int stride, int pad, at::Tensor y, int ldy, int yoff,
                            const at::Tensor& z, int ldz, int zoff, const at::Tensor& mscale,
                            const at::Tensor& mshift) {
  require_gpu(x, "x");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  ConvArgs a{};
  a.f32 = act_f32(x, "conv2d_fwd_bnbwd");
  same_type(x, w, "conv2d_fwd_bnbwd w");
  same_type(x, z, "conv2d_fwd_bnbwd z");
  same_type(x, y, "conv2d_fwd_bnbwd y");
  a.x = ptr<uint16_t>(x);
  a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.xoff = xoff;
  a.w = ptr<uint16_t>(w);
  a.ldw = R * S * C;
  a.S = S;
  a.OH = P; a.OW = Q;
  a.so = 1; a.sa = stride;
  a.Nimg = N; a.Kout = K;
  fill_epilogue(a, y, ldy, yoff, c10::nullopt, c10::nullopt, 0, 0, c10::nullopt, c10::nullopt, false, c10::nullopt);
  a.vec_store = ((ldy % 8) == 0 && (yoff % 8) == 0) ? 1 : 0;
  a.z = ptr<uint16_t>(z);
  a.ldz = ldz; a.zoff = zoff;
  a.mscale = ptr<float>(mscale);
  a.mshift = ptr<float>(mshift);
  a.nstat = 2;
  if ((ldz | zoff) % 8 != 0 || !a.vec_store || K % 8)
    throw std::runtime_error("conv2d_fwd_bnbwd: fused BN tensors must be 8-channel aligned");
  set_kstep(a, C);
  int bm, bn;
  pick_tiles((int64_t)N * P * Q, K, (int64_t)R * S * C, C, bm, bn);
  if (a.f32) f32_tiles(bm, bn);
  const int pipe = pipe_select(a.f32, 0, C, (int64_t)N * P * Q, K, (int64_t)R * S * C, bm, bn);
  a.ntiles = ceil_div(K, bn);
  a.nphase = 1;
  ConvPhase& p = a.ph[0];
  p.P = P; p.Q = Q; p.Tr = R; p.Ts = S;
  p.dh0 = -pad; p.dhs = 1; p.dw0 = -pad; p.dws = 1;
  p.wr0 = 0; p.wrs = 1; p.ws0 = 0; p.wss = 1;
  p.oh0 = 0; p.ow0 = 0;
  finish_phase(p, N, C, bm, a.f32);
  at::Tensor stats = at::empty({(int64_t)p.mtiles, 2, (int64_t)K}, x.options().dtype(at::kFloat));
  a.stats = ptr<float>(stats);
  if (g_splitk_override > 0) a.splitk_req = g_splitk_override;
  check(dlmpi_conv_igemm_ex(&a, bm, bn, pipe, cur_stream()), "conv2d_fwd_bnbwd");
  return stats;
}

// Number of BN-stat partial rows conv2d_fwd will produce (so the caller can size `stats`).
int conv2d_fwd_mtiles_pro(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int bm_req, int pro,
                          int f32) {
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  int bm, bn;
  if (pro == 3) return ceil_div((int64_t)N * P * Q, kPro3Bm);   // either pro-3 path (apply_kernel)
  // The rows of the tiled (conv_igemm / pipe / halo) launch ...
  const int general = [&]() -> int {
    if (bm_req <= 0) {
      int hbm, hbn;
      pick_tiles((int64_t)N * P * Q, K, (int64_t)R * S * C, C, hbm, hbn, pro != 0);
      if (f32) f32_tiles(hbm, hbn);
      const bool halo_ok = halo_eligible(f32, pro, C, R, S, stride, pad, P, Q);
      if (!halo_first(halo_ok, K) && pipe_select(f32, pro, C, (int64_t)N * P * Q, K, (int64_t)R * S * C, hbm, hbn))
        return ceil_div((int64_t)N * P * Q, hbm);
      if (halo_ok) return halo_mtiles(N, P, Q, K, hbn);
    }
    // autotuned launches may pick any M tile: size for the smallest (64 rows)
    if (bm_req <= 0 && conv_autotune_on() && !f32 && pro == 0) return ceil_div((int64_t)N * P * Q, 64);
    pick_tiles((int64_t)N * P * Q, K, (int64_t)R * S * C, C, bm, bn, pro != 0);
    if (f32) f32_tiles(bm, bn);
    if (bm_req > 0) bm = bm_req;
    return ceil_div((int64_t)N * P * Q, bm);
  }();
  // ... and, where a persistent kernel is planned (one statistics row per block), the larger of the
  // two: its launch conditions on strides / offsets / storage are checked at launch time, and when one
  // fails the forward takes the tiled path into the same buffer
  int G, th, tw;
  if (bm_req <= 0 && c8_shape((int64_t)N * H * W, C, K, R, S, stride, pad, W, pro, f32, G)) return std::max(G, general);
  if (bm_req <= 0 && c16_shape(N, H, W, C, K, R, S, stride, pad, pro, f32, G)) return std::max(G, general);
  if (bm_req <= 0 && stream1x1_shape((int64_t)N * P * Q, C, K, R, S, stride, pad, pro, f32, bm, bn, G))
    return std::max(G, general);
  if (bm_req <= 0 && stream3x3_shape(N, H, W, C, K, R, S, stride, pad, pro, f32, th, tw, G)) return std::max(G, general);
  return general;
}
int conv2d_fwd_mtiles(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int bm_req) {
  return conv2d_fwd_mtiles_pro(N, H, W, C, K, R, S, stride, pad, bm_req, 0, 0);
}

// dx[n, h, w, dxoff + c] = sum_{r,s,k} dy[n, (h+pad-r)/stride, (w+pad-s)/stride, k] * wT[c][r][s][k]  (+ res)
// as stride^2 dense sub-pixel phases.
//
// Optional BN-backward fusion (dx is the gradient of y = relu(BN(z)) [+ BN2(z2)]): the epilogue
// applies the ReLU mask [y > 0] before storing and emits per-tile partials
// [tiles][2|3][C] = {sum dx, sum dx*z [, sum dx*z2]}, returned (None without z).
c10::optional<at::Tensor> conv2d_dgrad_pro(const at::Tensor& dy, int N, int P, int Q, int K, int lddy, int dyoff,
                                       const at::Tensor& wT, int C, int R, int S, int stride, int pad, int H, int W,
                                       at::Tensor dx, int lddx, int dxoff, const c10::optional<at::Tensor>& res,
                                       int ldres, int resoff, const c10::optional<at::Tensor>& mask, int ldmask,
                                       int maskoff, const c10::optional<at::Tensor>& z, int ldz, int zoff,
                                       const c10::optional<at::Tensor>& z2, int ldz2, int z2off,
                                       const c10::optional<at::Tensor>& mscale,
                                       const c10::optional<at::Tensor>& mshift,
                                       const c10::optional<at::Tensor>& mbits, bool colsum, int pro,
                                       const c10::optional<at::Tensor>& pk0, const c10::optional<at::Tensor>& pk1,
                                       const c10::optional<at::Tensor>& pz, int ldpz, int pzoff,
                                       const c10::optional<at::Tensor>& bias) {
  require_gpu(dy, "dy");
  if (stride > 2) throw std::runtime_error("conv2d_dgrad: stride <= 2 supported");
  if (bias.has_value() && bias->defined() && (bias->scalar_type() != at::kFloat || bias->numel() < C))
    throw std::runtime_error("conv2d_dgrad: bias must be fp32 [C]");
  ConvArgs a{};
  a.f32 = act_f32(dy, "conv2d_dgrad");
  same_type(dy, wT, "conv2d_dgrad wT");
  same_type(dy, dx, "conv2d_dgrad dx");
  same_type(dy, res, "conv2d_dgrad res");
  same_type(dy, mask, "conv2d_dgrad mask");
  same_type(dy, z, "conv2d_dgrad z");
  same_type(dy, z2, "conv2d_dgrad z2");
  a.x = ptr<uint16_t>(dy);
  a.H = P; a.W = Q; a.C = K; a.ldx = lddy; a.xoff = dyoff;
  a.w = ptr<uint16_t>(wT);
  a.ldw = R * S * K;
  a.S = S;
  a.OH = H; a.OW = W;
  a.so = stride; a.sa = 1;
  a.Nimg = N; a.Kout = C;
  fill_epilogue(a, dx, lddx, dxoff, bias, res, ldres, resoff, c10::nullopt, c10::nullopt, false, c10::nullopt);
  a.vec_store = ((lddx % 8) == 0 && (dxoff % 8) == 0) ? 1 : 0;
  a.mask = optr<uint16_t>(mask);
  a.ldmask = ldmask; a.maskoff = maskoff;
  a.z = optr<uint16_t>(z);
  a.ldz = ldz; a.zoff = zoff;
  a.z2 = optr<uint16_t>(z2);
  a.ldz2 = ldz2; a.z2off = z2off;
  a.mscale = optr<float>(mscale);
  a.mshift = optr<float>(mshift);
  a.mbits = optr<uint8_t>(mbits);
  if (a.mbits && (mbits->numel() != (int64_t)N * H * W * (C / 8) || C % 8))
    throw std::runtime_error("conv2d_dgrad: mask bits must be [N*H*W][C/8]");
  a.nstat = a.z2 ? 3 : 2;
  if (a.z && !a.mask && !a.mscale && !a.mbits)
    throw std::runtime_error("conv2d_dgrad: fused BN statistics need the ReLU mask");
  if (a.mscale && (!a.z || !a.mshift)) throw std::runtime_error("conv2d_dgrad: mask from z needs z, scale, shift");
  if ((a.mask || a.mscale || a.mbits) && ((ldmask | maskoff | ldz | zoff | ldz2 | z2off) % 8 != 0 || !a.vec_store))
    throw std::runtime_error("conv2d_dgrad: fused BN tensors must be 8-channel aligned");
  g_dgrad_stream_ran = 0;
  g_conv3_ran = 0;
  {  // streaming 3x3 data gradient (conv3x3_stream.hip, 64 -> 64): a forward conv of dy with wT, taps flipped
    const int mode = a.mscale ? 2 : 0;
    int th, tw, G;
    if (stream3x3_shape(N, H, W, K, C, R, S, stride, pad, pro, a.f32, th, tw, G) && P == H && Q == W && !colsum &&
        !a.mask && !a.mbits && !a.z2 && !a.res && !a.bias && (a.z != nullptr) == (mode == 2) && a.vec_store &&
        a.kvalid == C && (lddy | dyoff) % 8 == 0 && (int64_t)H * W * lddx * 2 < (1ll << 31) &&
        dx.scalar_type() == at::kBFloat16) {
      dlmpi::Conv3StreamArgs c = conv3_args(dy, N, H, W, lddy, dyoff, wT, 1, a.y, lddx, dxoff, th, tw, G);
      c.z = static_cast<const uint16_t*>(a.z);
      c.ldz = ldz; c.zoff = zoff;
      c.mscale = a.mscale; c.mshift = a.mshift;
      c10::optional<at::Tensor> st;
      if (a.z) {
        st = at::empty({(int64_t)G, 2, (int64_t)C}, dy.options().dtype(at::kFloat));
        c.stats = ptr<float>(*st);
      }
      check(dlmpi_conv3x3_stream(&c, mode == 2 ? 2 : 1, cur_stream()), "conv2d_dgrad (stream 3x3)");
      g_conv3_ran = 1;
      return st;
    }
  }
  {  // streaming 1x1 data gradient (conv1x1_dgrad_stream.hip): memory-bound GEMMs with a heavy epilogue
    const int64_t M = (int64_t)N * H * W;
    const int mode = a.mbits ? 1 : (a.mscale ? 2 : 0);
    int sbm, sbn, G;
    const auto fits = [](int64_t rows, int64_t ld) { return rows * ld < (1ll << 31); };
    if (R == 1 && S == 1 && stride == 1 && pad == 0 && !a.f32 && pro == 0 && !colsum && !a.mask &&
        (a.z != nullptr) == (mode != 0) && a.vec_store && a.kvalid == C && (lddy | dyoff) % 8 == 0 &&
        (!a.res || (ldres | resoff) % 8 == 0) && fits(M, lddy) && fits(M, lddx) && (!a.res || fits(M, ldres)) &&
        (!a.z || fits(M, ldz)) && (!a.z2 || fits(M, ldz2)) && dx.scalar_type() == at::kBFloat16 &&
        dlmpi_dgrad_stream_plan(M, K, C, mode, a.z2 ? 1 : 0, a.res ? 1 : 0, &sbm, &sbn, &G)) {
      DgradStreamArgs sa{};
      sa.x = ptr<uint16_t>(dy);
      sa.ldx = lddy; sa.xoff = dyoff;
      sa.w = ptr<uint16_t>(wT);
      sa.y = reinterpret_cast<uint16_t*>(a.y);
      sa.ldy = lddx; sa.yoff = dxoff;
      sa.y_bytes = (int)std::min<int64_t>(INT32_MAX, (int64_t)dx.numel() * 2);
      sa.M = (int)M; sa.K = K; sa.Kout = C;
      sa.bias = a.bias;
      sa.res = static_cast<const uint16_t*>(a.res);
      sa.ldres = ldres; sa.resoff = resoff;
      sa.z = static_cast<const uint16_t*>(a.z);
      sa.ldz = ldz; sa.zoff = zoff;
      sa.z2 = static_cast<const uint16_t*>(a.z2);
      sa.ldz2 = ldz2; sa.z2off = z2off;
      sa.mbits = a.mbits;
      sa.mscale = a.mscale; sa.mshift = a.mshift;
      sa.G = G; sa.ntiles = C / sbn; sa.mtiles = (int)ceil_div(M, sbm);
      c10::optional<at::Tensor> st;
      if (a.z) {
        st = at::empty({(int64_t)G, (int64_t)a.nstat, (int64_t)C}, dy.options().dtype(at::kFloat));
        sa.stats = ptr<float>(*st);
      }
      check(dlmpi_conv1x1_dgrad_stream(&sa, sbm, sbn, mode, cur_stream()), "conv2d_dgrad (stream 1x1)");
      g_dgrad_stream_ran = 1;
      return st;
    }
  }
  set_kstep(a, K);
  set_prologue(a, pro, pk0, pk1, pz, ldpz, pzoff);
  int bm, bn;
  pick_tiles((int64_t)N * H * W / (stride * stride), C, (int64_t)R * S * K / (stride * stride), K, bm, bn, pro != 0);
  if (a.f32) f32_tiles(bm, bn);
  const bool halo_ok = halo_eligible(a.f32, pro, K, R, S, stride, pad, H, W) && P == H && Q == W;
  const int pipe = halo_first(halo_ok, C) || g_pipe_dgrad_override == 0
                       ? 0 : pipe_select(a.f32, pro, K, (int64_t)N * H * W / (stride * stride), C,
                                         (int64_t)R * S * K / (stride * stride), bm, bn);
  const bool halo = !pipe && halo_ok;
  if (halo) halo_tiles(C, bm, bn);
  a.ntiles = ceil_div(C, bn);
  a.nphase = stride * stride;
  int tiles = 0;
  for (int ph = 0; ph < stride; ++ph) {
    for (int pw = 0; pw < stride; ++pw) {
      ConvPhase& p = a.ph[ph * stride + pw];
      const int r0 = (ph + pad) % stride, s0 = (pw + pad) % stride;
      p.P = (H - ph + stride - 1) / stride;
      p.Q = (W - pw + stride - 1) / stride;
      p.Tr = r0 < R ? (R - r0 + stride - 1) / stride : 0;
      p.Ts = s0 < S ? (S - s0 + stride - 1) / stride : 0;
      p.dh0 = (ph + pad - r0) / stride; p.dhs = -1;
      p.dw0 = (pw + pad - s0) / stride; p.dws = -1;
      p.wr0 = r0; p.wrs = stride; p.ws0 = s0; p.wss = stride;
      p.oh0 = ph; p.ow0 = pw;
      finish_phase(p, N, K, bm, a.f32);
      p.tile_base = tiles;
      tiles += p.mtiles;
    }
  }
  if (halo) {
    apply_halo(a, N, bm);
    tiles = a.ph[0].mtiles;
  }
  g_halo_ran = halo ? 1 : 0;
  {  // autotuned tiling (statistics: a placeholder until the tile count is known -- the trials
     // write to scratch)
    const bool want_stats = a.z || colsum;
    a.stats = want_stats ? reinterpret_cast<float*>(static_cast<uintptr_t>(256)) : nullptr;
    if (!pipe && conv_plan(a, 1, bm, bn)) {
      tiles = 0;
      for (int i = 0; i < a.nphase; ++i) tiles += a.ph[i].mtiles;
    }
    a.stats = nullptr;
  }
  c10::optional<at::Tensor> stats;
  if (a.z || colsum) {
    // colsum without BN fusion: per-tile {sum dx, sum dx^2} of the stored gradient (UNet: the
    // column sums of the up-sampling slice are the ConvTranspose2d bias gradient)
    stats = at::empty({(int64_t)tiles, (int64_t)a.nstat, (int64_t)C}, dy.options().dtype(at::kFloat));
    a.stats = ptr<float>(*stats);
  }
  if (g_splitk_override > 0) a.splitk_req = g_splitk_override;
  check(dlmpi_conv_igemm_ex(&a, bm, bn, pipe, cur_stream()), "conv2d_dgrad");
  return stats;
}

c10::optional<at::Tensor> conv2d_dgrad(const at::Tensor& dy, int N, int P, int Q, int K, int lddy, int dyoff,
                                       const at::Tensor& wT, int C, int R, int S, int stride, int pad, int H, int W,
                                       at::Tensor dx, int lddx, int dxoff, const c10::optional<at::Tensor>& res,
                                       int ldres, int resoff, const c10::optional<at::Tensor>& mask, int ldmask,
                                       int maskoff, const c10::optional<at::Tensor>& z, int ldz, int zoff,
                                       const c10::optional<at::Tensor>& z2, int ldz2, int z2off,
                                       const c10::optional<at::Tensor>& mscale,
                                       const c10::optional<at::Tensor>& mshift,
                                       const c10::optional<at::Tensor>& mbits, bool colsum) {
  return conv2d_dgrad_pro(dy, N, P, Q, K, lddy, dyoff, wT, C, R, S, stride, pad, H, W, dx, lddx, dxoff, res, ldres,
                          resoff, mask, ldmask, maskoff, z, ldz, zoff, z2, ldz2, z2off, mscale, mshift, mbits, colsum,
                          0, c10::nullopt, c10::nullopt, c10::nullopt, 0, 0, c10::nullopt);
}

// ConvTranspose2d(k=2, s=2): y[n, 2h+i, 2w+j, yoff + co] = bias[co] + sum_ci x[n,h,w,ci] * wf[co][i][j][ci]
void convT2x2_fwd(const at::Tensor& x, int N, int H, int W, int Cin, int ldx, int xoff, const at::Tensor& wf, int Cout,
                  at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& bias) {
  require_gpu(x, "x");
  ConvArgs a{};
  a.f32 = act_f32(x, "convT2x2_fwd");
  same_type(x, wf, "convT2x2_fwd w");
  same_type(x, y, "convT2x2_fwd y");
  a.x = ptr<uint16_t>(x);
  a.H = H; a.W = W; a.C = Cin; a.ldx = ldx; a.xoff = xoff;
  a.w = ptr<uint16_t>(wf);
  a.ldw = 4 * Cin;
  a.S = 2;
  a.OH = 2 * H; a.OW = 2 * W;
  a.so = 2; a.sa = 1;
  a.Nimg = N; a.Kout = Cout;
  fill_epilogue(a, y, ldy, yoff, bias, c10::nullopt, 0, 0, c10::nullopt, c10::nullopt, false, c10::nullopt);
  a.vec_store = ((ldy % 8) == 0 && (yoff % 8) == 0) ? 1 : 0;
  set_kstep(a, Cin);
  g_convT_stream_ran = 0;
  {  // the streaming 1x1 kernel over 4 Cout columns (input read once for the four sub-pixel positions)
    const int64_t M = (int64_t)N * H * W;
    int sbm, sbn, G;
    // (output offsets are relative to each tile's first output row: any buffer size; input 32-bit)
    if (g_convT_stream && !a.f32 && a.vec_store && ldx % 8 == 0 && xoff % 8 == 0 && M * ldx < (1ll << 31) &&
        4 * (int64_t)W * ldy * 2 * 4 < (1ll << 31) && 4 * M < (1ll << 31) &&
        dlmpi_stream1x1_plan(M, Cin, 4 * Cout, 1, &sbm, &sbn, &G) && Cout % sbn == 0) {
      Stream1x1Args sa{};
      sa.x = ptr<uint16_t>(x);
      sa.ldx = ldx; sa.xoff = xoff;
      sa.w = ptr<uint16_t>(wf);
      sa.y = reinterpret_cast<uint16_t*>(a.y);
      sa.ldy = ldy; sa.yoff = yoff;
      sa.y_bytes = (int)std::min<int64_t>(INT32_MAX, (int64_t)y.numel() * 2);   // (UP2: per-tile descriptors)
      sa.M = (int)M; sa.C = Cin; sa.Kout = 4 * Cout;
      sa.bias = a.bias;
      sa.G = G; sa.ntiles = 4 * Cout / sbn; sa.mtiles = ceil_div(M, sbm);
      sa.H = H; sa.W = W;
      sa.fdPQ = make_fastdiv((uint32_t)(H * W));
      sa.fdQ = make_fastdiv((uint32_t)W);
      sa.up2 = 1; sa.Cup = Cout;
      check(dlmpi_conv1x1_stream(&sa, sbm, sbn, cur_stream()), "convT2x2_fwd (stream)");
      g_convT_stream_ran = 1;
      return;
    }
  }
  int bm, bn;
  pick_tiles((int64_t)N * H * W, Cout, Cin, Cin, bm, bn, false, false);   // 4-phase convT: unmeasured at 256 rows
  if (a.f32) f32_tiles(bm, bn);
  a.ntiles = ceil_div(Cout, bn);
  a.nphase = 4;
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) {
      ConvPhase& p = a.ph[i * 2 + j];
      p.P = H; p.Q = W; p.Tr = 1; p.Ts = 1;
      p.dh0 = 0; p.dhs = 0; p.dw0 = 0; p.dws = 0;
      p.wr0 = i; p.wrs = 0; p.ws0 = j; p.wss = 0;
      p.oh0 = i; p.ow0 = j;
      finish_phase(p, N, Cin, bm, a.f32);
    }
  check(dlmpi_conv_igemm(&a, bm, bn, cur_stream()), "convT2x2_fwd");
}

// grad[ko][t][c] += sum_pix dy[pix][dyoff + ko] * x[gather(pix, t)][xoff + c]   (c < Creal, ko < Ko_real)
// dy is over the P x Q output grid of a conv (R x S, stride, pad) applied to x (H x W).
// Operand prologues: pro_a 2 -> the dy operand is dz = pcoef[0] dy + pcoef[1] Z + pcoef[2] (a deferred
// BN-backward apply, Z = the BN input); pro_b 1 -> the x operand is relu(x * pscale + pshift).
// ---- deferred weight-gradient split reductions --------------------------------------------------
// With set_wgrad_defer(1) (the engine backward) a weight gradient's split reduction is queued instead
// of launched; wgrad_flush() -- the DDP reducer before each bucket launch, the engine at the end of its
// backward, and a full queue (kWgradBatch entries) -- launches the queue as two batched kernels
// (conv_wgrad.hip wgrad_reduce_batch_s1/s2: the same sums in the same order as dlmpi_wgrad_reduce's
// two launches per gradient) on the current stream.  Queued entries keep their slab tensors alive; an entry queued on
// another stream is ordered before the flush by an event, and its slab's reuse by recordStream.
struct PendingReduce {
  at::Tensor ws;
  hipStream_t s;
  dlmpi::WgradReduceEntry e;
};
static std::vector<PendingReduce> g_pending;
static bool g_wgrad_defer = false;
static int g_wgrad_batch = dlmpi::kWgradBatch;   // queue length that triggers a flush (A/B: set_wgrad_batch)
static bool g_defer_direct = true;               // also queue the one-launch (G == 0) reductions (A/B)
static bool g_wgrad_bypass = false;              // reduce the next weight gradients immediately, queue kept
static int64_t g_reduce_launches = 0;   // reduction launches (either form), for tests / bench

// Launches the queue.  The queue is moved out first: if a launch throws midway, the batches already
// launched are not launched (and added into the gradients) a second time by a later flush, and the
// rest are dropped with the step that failed.
void wgrad_flush() {
  if (g_pending.empty()) return;
  std::vector<PendingReduce> pending;
  pending.swap(g_pending);
  const hipStream_t cur = cur_stream();
  std::vector<hipStream_t> waited;
  for (auto& p : pending) {
    if (p.s == cur) continue;
    if (std::find(waited.begin(), waited.end(), p.s) == waited.end()) {
      hipEvent_t ev;
      check(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "wgrad_flush event");
      check(hipEventRecord(ev, p.s), "wgrad_flush record");
      check(hipStreamWaitEvent(cur, ev, 0), "wgrad_flush wait");
      check(hipEventDestroy(ev), "wgrad_flush event");
      waited.push_back(p.s);
    }
    c10::hip::HIPCachingAllocator::recordStream(p.ws.storage().data_ptr(), c10::hip::getCurrentHIPStream());
  }
  dlmpi::WgradReduceBatch b{};
  bool two = false;
  for (size_t i = 0; i < pending.size(); ++i) {
    const dlmpi::WgradReduceEntry& e = pending[i].e;
    two |= e.splits > 1 && dlmpi_wgrad_reduce_groups(e.splits, e.total) > 0;
    b.e[b.n++] = e;
    if (b.n == g_wgrad_batch || i + 1 == pending.size()) {
      check(dlmpi_wgrad_reduce_batch(&b, cur), "wgrad_reduce_batch");
      g_reduce_launches += two ? 2 : 1;
      b.n = 0;
      two = false;
    }
  }
}

// Drops the queue without launching it and turns deferral off: the backward that queued it failed
// (e.g. a hipGraph capture torn down mid-backward: its slabs were never computed and its streams are
// abandoned).  The engine's error path and CapturedStep's stream reset call it.
void wgrad_discard() {
  g_pending.clear();
  g_wgrad_defer = false;
  g_wgrad_bypass = false;
}

// the split reduction of a weight gradient: ws = [splits + G][wsz] (G = dlmpi_wgrad_reduce_groups)
static void wgrad_reduce_or_defer(const at::Tensor& ws, int splits, int G, int64_t wsz, int Ko, int T, int Cpad,
                                  int Creal, int Ko_real, at::Tensor& grad) {
  float* out = ptr<float>(grad);
  for (const auto& p : g_pending)   // a gradient accumulated twice: its first sum goes out first
    if (p.e.out == out) {
      wgrad_flush();
      break;
    }
  if (!g_wgrad_defer || g_wgrad_bypass || (!g_defer_direct && !(splits > 1 && G > 0))) {
    check(dlmpi_wgrad_reduce(ptr<float>(ws), splits, Ko, T, Cpad, Creal, Ko_real, out, ptr<float>(ws) + (int64_t)splits * wsz,
                             (int)std::min<int64_t>(INT32_MAX, (int64_t)G * wsz), cur_stream()),
          "wgrad_reduce");
    g_reduce_launches += splits > 1 && G > 0 ? 2 : 1;
    return;
  }
  if (Ko_real == 0 || wsz == 0) return;
  PendingReduce p{ws, cur_stream(), {}};
  p.e.ws = ptr<float>(ws);
  p.e.ws2 = G > 0 ? ptr<float>(ws) + (int64_t)splits * wsz : nullptr;
  p.e.out = out;
  p.e.total = (int64_t)Ko * T * Cpad;
  p.e.splits = splits;
  p.e.Ko_real = Ko_real;
  p.e.T = T;
  p.e.Cpad = Cpad;
  p.e.Creal = Creal;
  g_pending.push_back(std::move(p));
  if ((int)g_pending.size() >= g_wgrad_batch) wgrad_flush();
}

static int g_wgrad3_override = -1;   // dlmpi_ext set_wgrad3 (tests); -1: on
static int g_wgrad3_blocks = 0;      // dlmpi_ext set_wgrad3_blocks (A/B): > 0 overrides the grid target
static int g_wgrad3_ran = 0;         // 1 if the last weight gradient ran the 3x3 spatial-tile kernel
static int g_wgrad_blocks = 0;       // dlmpi_ext set_wgrad_blocks (A/B): > 0 overrides the gather kernel's grid target

void conv2d_wgrad_pro(const at::Tensor& dy, int lddy, int dyoff, int Ko, const at::Tensor& x, int N, int H, int W,
                      int C, int ldx, int xoff, int R, int S, int stride, int pad, int P, int Q, at::Tensor grad,
                      int Creal, int Ko_real, int pro_a, const c10::optional<at::Tensor>& pcoef,
                      const c10::optional<at::Tensor>& pz, int ldpz, int pzoff, int pro_b,
                      const c10::optional<at::Tensor>& pscale, const c10::optional<at::Tensor>& pshift) {
  require_gpu(dy, "dy");
  if (C % 8 != 0 || Ko % 8 != 0) throw std::runtime_error("conv2d_wgrad: channels must be multiples of 8");
  WgradArgs a{};
  a.f32 = act_f32(dy, "conv2d_wgrad");
  same_type(dy, x, "conv2d_wgrad x");
  if (a.f32 && (pro_a || pro_b)) throw std::runtime_error("conv2d_wgrad: operand prologues are bf16 only");
  a.pro_a = pro_a;
  a.pro_b = pro_b;
  if (pro_a) {
    a.pcoef = optr<float>(pcoef);
    a.pz = optr<uint16_t>(pz);
    a.ldpz = ldpz;
    a.pzoff = pzoff;
    if (pro_a != 2 || !a.pcoef || !a.pz || pcoef->numel() < 3 * Ko || (ldpz | pzoff) % 8)
      throw std::runtime_error("conv2d_wgrad: prologue a needs coef [3][Ko] and an aligned Z");
  }
  if (pro_b) {
    a.pscale = optr<float>(pscale);
    a.pshift = optr<float>(pshift);
    if (pro_b != 1 || !a.pscale || !a.pshift || pscale->numel() < C || pshift->numel() < C)
      throw std::runtime_error("conv2d_wgrad: prologue b needs scale / shift of C channels");
  }
  // 3x3 / stride 1 / pad 1 without operand prologues (UNet DoubleConv, ResNet conv2): the
  // spatial-tile kernel (conv_wgrad3.hip) -- X staged once per 8 x 8 pixel block for all 9 taps.
  int kt = 0, ct = 0;
  // Only where the 8 x 8 blocks are at least 3/4 full: 14^2 / 7^2 are (77 %), the 4^2 / 2^2 / 1^2 images
  // of ResNet-18 on 32^2 CIFAR are not (25 % / 6 % / 2 %) and take the gather kernel.
  const bool w3_full = 4 * H * W >= 3 * ceil_div(H, 8) * 8 * ceil_div(W, 8) * 8;
  if (g_wgrad3_override != 0 && (w3_full || g_wgrad3_override == 1) && !a.f32 && pro_a == 0 && pro_b == 0 &&
      R == 3 && S == 3 && stride == 1 && pad == 1 && P == H && Q == W && dlmpi_wgrad3_plan(Ko, C, &kt, &ct)) {
    dlmpi::Wgrad3Args b{};
    b.dy = ptr<uint16_t>(dy);
    b.ldy = lddy; b.dyoff = dyoff; b.Ko = Ko;
    b.x = ptr<uint16_t>(x);
    b.ldx = ldx; b.xoff = xoff; b.C = C;
    b.H = H; b.W = W;
    b.tiles_h = ceil_div(H, 8);
    b.tiles_w = ceil_div(W, 8);
    b.ntiles_pix = N * b.tiles_h * b.tiles_w;
    b.mtiles = Ko / kt;
    b.ntiles = C / ct;
    // one 512-thread block per CU (252 VGPRs: 2 waves per SIMD take a SIMD's whole register file,
    // so nothing of the data-gradient chain on the main stream can share a CU with it).  Large
    // gradients (UNet, >= 64 G MAC) fill the chip once; the ResNet-size ones (~30 G MAC) leave ~100
    // CUs to the main stream (measured, profiles/r3_wgrad3: ResNet-50 12,233 img/s at 256 blocks vs
    // 12,348 at 160; UNet-512 470 vs 466).
    const double macs = (double)N * H * W * Ko * 9.0 * C;
    // (UNet-size gradients: 224 blocks leave 32 CUs to the data-gradient chain's small kernels, which
    // otherwise wait for the whole kernel -- UNet-512 +0.65 %, UNet-1024 +0.4 % over 256, 5 same-box
    // pairs, profiles/r4_unet)
    // (64 x 64 tiles are 4-wave blocks, two per CU: twice the blocks for the same CUs)
    const int target = (g_wgrad3_blocks > 0 ? g_wgrad3_blocks : (macs >= 64e9 ? 224 : 160)) * (kt == 64 && ct == 64 ? 2 : 1);
    const int kc = b.mtiles * b.ntiles;
    int splits = std::max(1, std::min(b.ntiles_pix, target / kc));
    b.tiles_per_split = ceil_div(b.ntiles_pix, splits);
    splits = ceil_div(b.ntiles_pix, b.tiles_per_split);
    b.splits = splits;
    const int64_t wsz = (int64_t)Ko * 9 * C;
    const int G = splits > 1 ? dlmpi_wgrad_reduce_groups(splits, wsz) : 0;
    at::Tensor ws = at::empty({(int64_t)(splits + G) * wsz}, dy.options().dtype(at::kFloat));
    b.ws = ptr<float>(ws);
    g_wgrad3_ran = 1;
    check(dlmpi_wgrad3x3(&b, kt, ct, cur_stream()), "conv2d_wgrad (3x3 tiles)");
    wgrad_reduce_or_defer(ws, splits, G, wsz, Ko, 9, C, Creal, Ko_real, grad);
    return;
  }
  g_wgrad3_ran = 0;
  a.dy = ptr<uint16_t>(dy);
  a.ldy = lddy; a.dyoff = dyoff; a.Ko = Ko;
  a.x = ptr<uint16_t>(x);
  a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.xoff = xoff;
  a.Nimg = N; a.P = P; a.Q = Q; a.S = S;
  a.stride_h = stride; a.stride_w = stride; a.pad_h = pad; a.pad_w = pad;
  a.TC = R * S * C;
  a.npix = N * P * Q;
  a.direct = (R == 1 && S == 1 && stride == 1 && pad == 0 && P == H && Q == W) ? 1 : 0;
  if (!dlmpi_wgrad_pro_ok(a.direct, pro_a, pro_b))
    throw std::runtime_error("conv2d_wgrad: operand prologues: one of them, x's only for 1x1 gradients");
  const int bm = a.f32 || Ko <= 64 ? 64 : 128;   // fp32: conv_wgrad_f32_kernel's 64 x 64 tile
  a.mtiles = ceil_div(Ko, bm);
  // Ko <= 64 gather-form (3x3 / strided / stem) weight gradients: 64 x 256 tiles (1 x 4 waves of
  // 64 x 64) -- each dy row staged once per 256 columns, fewer LDS reads per MFMA.  The tile holds
  // ~200 VGPRs (2 blocks per CU), so its split count is floored to fit the grid in one round
  // (profiles/r2_wgrad_wide).  Gather-form only (1x1s measured no gain).
  const bool w256 = !a.f32 && Ko <= 64 && pro_b == 0 && a.TC >= 256 && !a.direct;
  const int bn = a.f32 ? 64 : (w256 ? 256 : 128);
  a.ntiles = ceil_div(a.TC, bn);
  const int tiles = a.mtiles * a.ntiles;
  // split the pixel reduction so the grid covers the chip ~2 blocks deep, but keep each split at
  // least 8 K-steps (512 pixels) so the fp32 slab traffic stays small next to the MFMA work.
  // target grid size (the weight gradients share the GPU with the data-gradient
  // chain on another stream, so they need not fill it alone)
  const int target_blocks = g_wgrad_blocks > 0 ? g_wgrad_blocks : 512;
  const int maxsplit = std::max(1, ceil_div(a.npix, 512));
  int splits = std::max(1, std::min(maxsplit, w256 ? target_blocks / tiles : ceil_div(target_blocks, tiles)));
  int pps = ceil_div(a.npix, splits);
  pps = ceil_div(pps, 64) * 64;
  splits = ceil_div(a.npix, pps);
  a.splits = splits;
  a.pix_per_split = pps;
  a.fdPQ = make_fastdiv((uint32_t)(P * Q));
  a.fdQ = make_fastdiv((uint32_t)Q);
  a.fdC = make_fastdiv((uint32_t)C);
  a.fdS = make_fastdiv((uint32_t)S);
  const int64_t wsz = (int64_t)Ko * a.TC;
  const int G = splits > 1 ? dlmpi_wgrad_reduce_groups(splits, wsz) : 0;
  at::Tensor ws = at::empty({(int64_t)(splits + G) * wsz}, dy.options().dtype(at::kFloat));
  a.ws = ptr<float>(ws);
  check(dlmpi_conv_wgrad(&a, bm, bn, cur_stream()), "conv2d_wgrad");
  wgrad_reduce_or_defer(ws, splits, G, wsz, Ko, R * S, C, Creal, Ko_real, grad);
}

void conv2d_wgrad(const at::Tensor& dy, int lddy, int dyoff, int Ko, const at::Tensor& x, int N, int H, int W, int C,
                  int ldx, int xoff, int R, int S, int stride, int pad, int P, int Q, at::Tensor grad, int Creal,
                  int Ko_real) {
  conv2d_wgrad_pro(dy, lddy, dyoff, Ko, x, N, H, W, C, ldx, xoff, R, S, stride, pad, P, Q, grad, Creal, Ko_real, 0,
                   c10::nullopt, c10::nullopt, 0, 0, 0, c10::nullopt, c10::nullopt);
}

static at::Tensor colsum_ws(const at::Tensor& like, int T, int C) {
  return at::empty({(int64_t)dlmpi_colsum_ws_doubles(T, C)}, like.options().dtype(at::kDouble));
}

// --------------------------------- batch norm ----------------------------------------------
void bn_finalize(const at::Tensor& partial, int ntiles, int C, double count, const c10::optional<at::Tensor>& gamma,
                 const c10::optional<at::Tensor>& beta, const c10::optional<at::Tensor>& running_mean,
                 const c10::optional<at::Tensor>& running_var, double momentum, double eps, at::Tensor scale,
                 at::Tensor shift, const c10::optional<at::Tensor>& save_mean,
                 const c10::optional<at::Tensor>& save_invstd) {
  at::Tensor ws = colsum_ws(partial, ntiles, C);
  check(dlmpi_bn_finalize(ptr<float>(partial), ntiles, C, count, optr<float>(gamma), optr<float>(beta),
                          optr<float>(running_mean), optr<float>(running_var), (float)momentum, (float)eps,
                          ptr<float>(scale), ptr<float>(shift), optr<float>(save_mean), optr<float>(save_invstd),
                          ptr<double>(ws), cur_stream()),
        "bn_finalize");
}

int reduce_blocks(int64_t M, int C) { return dlmpi_reduce_blocks(M, C); }

void bn_stats(const at::Tensor& x, int64_t M, int C, int ldx, int xoff, at::Tensor partial, int nblk) {
  check(dlmpi_bn_stats(x.data_ptr(), M, C, ldx, xoff, ptr<float>(partial), nblk, act_f32(x, "bn_stats"), cur_stream()),
        "bn_stats");
}

void bn_apply(const at::Tensor& x, int ldx, int xoff, int64_t M, int C, const at::Tensor& scale,
              const at::Tensor& shift, const c10::optional<at::Tensor>& res, int ldres, int resoff, bool relu,
              at::Tensor y, int ldy, int yoff, const c10::optional<at::Tensor>& mbits,
              const c10::optional<at::Tensor>& rscale, const c10::optional<at::Tensor>& rshift) {
  if (mbits && mbits->numel() != M * (C / 8)) throw std::runtime_error("bn_apply: mask bits must be [M][C/8]");
  if (rscale.has_value() != rshift.has_value() || (rscale && !res))
    throw std::runtime_error("bn_apply: rscale / rshift come together, with a residual");
  if (rscale && (rscale->numel() < C || rshift->numel() < C)) throw std::runtime_error("bn_apply: rscale / rshift < C");
  same_type(x, y, "bn_apply y");
  same_type(x, res, "bn_apply res");
  check(dlmpi_bn_apply2(x.data_ptr(), ldx, xoff, M, C, ptr<float>(scale), ptr<float>(shift), optr<uint16_t>(res), ldres,
                        resoff, optr<float>(rscale), optr<float>(rshift), relu ? 1 : 0, y.data_ptr(), ldy, yoff,
                        optr<uint8_t>(mbits), act_f32(x, "bn_apply"), cur_stream()),
        "bn_apply");
}

void bn_bwd_reduce(const at::Tensor& dy, int lddy, int dyoff, const c10::optional<at::Tensor>& ymask, int ldym,
                   int ymoff, const c10::optional<at::Tensor>& x, int ldx, int xoff, int64_t M, int C,
                   const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& invstd, at::Tensor partial,
                   int nblk) {
  same_type(dy, ymask, "bn_bwd_reduce ymask");
  same_type(dy, x, "bn_bwd_reduce x");
  check(dlmpi_bn_bwd_reduce(dy.data_ptr(), lddy, dyoff, optr<uint16_t>(ymask), ldym, ymoff, optr<uint16_t>(x), ldx,
                            xoff, M, C, optr<float>(mean), optr<float>(invstd), ptr<float>(partial), nblk,
                            act_f32(dy, "bn_bwd_reduce"), cur_stream()),
        "bn_bwd_reduce");
}

void bn_bwd_finalize(const at::Tensor& partial, int nblk, int C, double count, const c10::optional<at::Tensor>& gamma,
                     const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& invstd,
                     const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
                     const c10::optional<at::Tensor>& coef) {
  at::Tensor ws = colsum_ws(partial, nblk, C);
  check(dlmpi_bn_bwd_finalize(ptr<float>(partial), nblk, C, count, optr<float>(gamma), optr<float>(mean),
                              optr<float>(invstd), optr<float>(dgamma), optr<float>(dbeta), optr<float>(coef),
                              ptr<double>(ws), cur_stream()),
        "bn_bwd_finalize");
}

// Finalize from the fused dgrad-epilogue partials [tiles][ns][C] (rows 0 and k2 = {sum dyr, sum dyr*z}).
void bn_bwd_finalize_fused(const at::Tensor& partial, int k2, int C, double count,
                           const c10::optional<at::Tensor>& gamma, const at::Tensor& mean, const at::Tensor& invstd,
                           const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
                           const c10::optional<at::Tensor>& coef) {
  const int T = (int)partial.size(0), ns = (int)partial.size(1);
  if (partial.size(2) != C) throw std::runtime_error("bn_bwd_finalize_fused: channel mismatch");
  at::Tensor ws = colsum_ws(partial, T, C);
  check(dlmpi_bn_bwd_finalize_ex(ptr<float>(partial), T, ns, k2, 1, C, count, optr<float>(gamma), ptr<float>(mean),
                                 ptr<float>(invstd), optr<float>(dgamma), optr<float>(dbeta), optr<float>(coef),
                                 ptr<double>(ws), cur_stream()),
        "bn_bwd_finalize_fused");
}

void bn_bwd_apply(const at::Tensor& dy, int lddy, int dyoff, const c10::optional<at::Tensor>& ymask, int ldym,
                  int ymoff, const at::Tensor& x, int ldx, int xoff, int64_t M, int C, const at::Tensor& coef,
                  at::Tensor dx, const c10::optional<at::Tensor>& dyr_out) {
  same_type(dy, ymask, "bn_bwd_apply ymask");
  same_type(dy, x, "bn_bwd_apply x");
  same_type(dy, dx, "bn_bwd_apply dx");
  same_type(dy, dyr_out, "bn_bwd_apply dyr_out");
  check(dlmpi_bn_bwd_apply(dy.data_ptr(), lddy, dyoff, optr<uint16_t>(ymask), ldym, ymoff, x.data_ptr(), ldx, xoff, M,
                           C, ptr<float>(coef), dx.data_ptr(), optr<uint16_t>(dyr_out), act_f32(dy, "bn_bwd_apply"),
                           cur_stream()),
        "bn_bwd_apply");
}

// w2 [C][2K] = {wT * coef[0], wT * coef[1]}, b [C] = wT . coef[2]: the dual 1x1 data gradient (bn.hip)
void dual_dgrad_weights(const at::Tensor& wT, int C, int K, const at::Tensor& coef, at::Tensor w2, at::Tensor b) {
  same_type(wT, w2, "dual_dgrad_weights w2");
  if (wT.numel() < (int64_t)C * K || w2.numel() < (int64_t)C * 2 * K || coef.numel() < 3 * (int64_t)K ||
      b.numel() < C || b.scalar_type() != at::kFloat || coef.scalar_type() != at::kFloat)
    throw std::runtime_error("dual_dgrad_weights: shapes / dtypes");
  check(dlmpi_dual_dgrad_weights(wT.data_ptr(), C, K, ptr<float>(coef), w2.data_ptr(), ptr<float>(b),
                                 act_f32(wT, "dual_dgrad_weights"), cur_stream()),
        "dual_dgrad_weights");
}

void channel_sum(const at::Tensor& x, int64_t M, int C, int ldx, int xoff, at::Tensor out_acc) {
  const int nblk = dlmpi_reduce_blocks(M, C);
  at::Tensor partial = at::empty({(int64_t)nblk * 2 * C}, x.options().dtype(at::kFloat));
  at::Tensor ws = colsum_ws(partial, nblk, C);
  check(dlmpi_channel_sum(x.data_ptr(), M, C, ldx, xoff, ptr<float>(out_acc), ptr<float>(partial), nblk,
                          ptr<double>(ws), act_f32(x, "channel_sum"), cur_stream()),
        "channel_sum");
}

// --------------------------------- pooling / layout ----------------------------------------
// ys (optional): also store the applied input relu(x * scale + shift) there (2x2 / s2 windows only)
void maxpool_fwd(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, int k, int stride, int pad,
                 at::Tensor y, at::Tensor idx, int OH, int OW, const c10::optional<at::Tensor>& scale,
                 const c10::optional<at::Tensor>& shift, const c10::optional<at::Tensor>& ys, int ldys, int ysoff) {
  same_type(x, y, "maxpool_fwd y");
  same_type(x, ys, "maxpool_fwd ys");
  check(dlmpi_maxpool_fwd(x.data_ptr(), N, H, W, C, ldx, xoff, k, stride, pad, y.data_ptr(), ptr<uint8_t>(idx), OH, OW,
                          optr<float>(scale), optr<float>(shift), ys.has_value() ? ys->data_ptr() : nullptr, ldys,
                          ysoff, act_f32(x, "maxpool_fwd"), cur_stream()),
        "maxpool_fwd");
}
void maxpool_bwd(const at::Tensor& dy, const at::Tensor& idx, int N, int H, int W, int C, int k, int stride, int pad,
                 int OH, int OW, const c10::optional<at::Tensor>& add, int ldadd, int addoff, at::Tensor dx, int lddx,
                 int dxoff) {
  same_type(dy, add, "maxpool_bwd add");
  same_type(dy, dx, "maxpool_bwd dx");
  check(dlmpi_maxpool_bwd(dy.data_ptr(), ptr<uint8_t>(idx), N, H, W, C, k, stride, pad, OH, OW, optr<uint16_t>(add),
                          ldadd, addoff, dx.data_ptr(), lddx, dxoff, act_f32(dy, "maxpool_bwd"), cur_stream()),
        "maxpool_bwd");
}
// data gradient of a 1x1 convolution with one output channel (UNet head) fused with the BN backward of
// the layer below; returns the partials [nblk][2][C] for bn_bwd_finalize_fused
at::Tensor outer_dgrad_bn(const at::Tensor& dy, int lddy, int64_t M, int C, const at::Tensor& w, int ldw,
                          const at::Tensor& z, const at::Tensor& mscale, const at::Tensor& mshift, at::Tensor dx) {
  require_gpu(dy, "dy");
  const int64_t rpb = 256 / (C / 8);
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(4096, (M + rpb * 8 - 1) / (rpb * 8)));
  at::Tensor part = at::empty({nblk, 2, C}, dy.options().dtype(at::kFloat));
  same_type(dy, w, "outer_dgrad_bn w");
  same_type(dy, z, "outer_dgrad_bn z");
  same_type(dy, dx, "outer_dgrad_bn dx");
  check(dlmpi_outer_dgrad_bn(dy.data_ptr(), lddy, M, C, w.data_ptr(), ldw, z.data_ptr(), ptr<float>(mscale),
                             ptr<float>(mshift), dx.data_ptr(), ptr<float>(part), nblk, act_f32(dy, "outer_dgrad_bn"),
                             cur_stream()),
        "outer_dgrad_bn");
  return part;
}
// max-pool backward fused with the BN-backward statistics of the producing BN+ReLU (mask from z);
// returns the partials [nblk][2][C] for bn_bwd_finalize_fused
at::Tensor maxpool_bwd_bn(const at::Tensor& dy, const at::Tensor& idx, int N, int H, int W, int C, int k, int stride,
                          int pad, int OH, int OW, const at::Tensor& z, const at::Tensor& mscale,
                          const at::Tensor& mshift, const c10::optional<at::Tensor>& add, int ldadd, int addoff,
                          at::Tensor dx) {
  // more blocks than the generic reductions: every row is a latency-bound window gather
  const int64_t rpb = 256 / (C / 8);
  const int nblk = (int)std::max<int64_t>(1, std::min<int64_t>(4096, ((int64_t)N * H * W + rpb * 8 - 1) / (rpb * 8)));
  at::Tensor part = at::empty({nblk, 2, C}, dy.options().dtype(at::kFloat));
  same_type(dy, z, "maxpool_bwd_bn z");
  same_type(dy, add, "maxpool_bwd_bn add");
  same_type(dy, dx, "maxpool_bwd_bn dx");
  check(dlmpi_maxpool_bwd_bn(dy.data_ptr(), ptr<uint8_t>(idx), N, H, W, C, k, stride, pad, OH, OW, z.data_ptr(),
                             ptr<float>(mscale), ptr<float>(mshift), optr<uint16_t>(add), ldadd, addoff, dx.data_ptr(),
                             ptr<float>(part), nblk, act_f32(dy, "maxpool_bwd_bn"), cur_stream()),
        "maxpool_bwd_bn");
  return part;
}
void avgpool_fwd(const at::Tensor& x, int N, int HW, int C, at::Tensor y) {
  same_type(x, y, "avgpool_fwd y");
  check(dlmpi_avgpool_fwd(x.data_ptr(), N, HW, C, y.data_ptr(), act_f32(x, "avgpool_fwd"), cur_stream()), "avgpool_fwd");
}
void avgpool_bwd(const at::Tensor& dy, int N, int HW, int C, at::Tensor dx) {
  same_type(dy, dx, "avgpool_bwd dx");
  check(dlmpi_avgpool_bwd(dy.data_ptr(), N, HW, C, dx.data_ptr(), act_f32(dy, "avgpool_bwd"), cur_stream()),
        "avgpool_bwd");
}
void nchw_to_nhwc(const at::Tensor& x, int N, int C, int H, int W, int Cpad, at::Tensor y) {
  check(dlmpi_nchw_to_nhwc(ptr<float>(x), N, C, H, W, Cpad, y.data_ptr(), act_f32(y, "nchw_to_nhwc"), cur_stream()),
        "nchw_to_nhwc");
}
void s2d_nchw(const at::Tensor& x, int N, int C, int H, int W, int pad, int U, int V, int CS, at::Tensor y) {
  check(dlmpi_s2d_nchw(ptr<float>(x), N, C, H, W, pad, U, V, CS, y.data_ptr(), act_f32(y, "s2d_nchw"), cur_stream()),
        "s2d_nchw");
}
void upsample2x_fwd(const at::Tensor& x, int N, int H, int W, int C, int ldx, int xoff, at::Tensor y, int ldy,
                    int yoff) {
  same_type(x, y, "upsample2x_fwd y");
  check(dlmpi_upsample2x_fwd(x.data_ptr(), N, H, W, C, ldx, xoff, y.data_ptr(), ldy, yoff, act_f32(x, "upsample2x_fwd"),
                             cur_stream()),
        "upsample2x_fwd");
}
void upsample2x_bwd(const at::Tensor& dy, int N, int H, int W, int C, int lddy, int dyoff, at::Tensor dx) {
  same_type(dy, dx, "upsample2x_bwd dx");
  check(dlmpi_upsample2x_bwd(dy.data_ptr(), N, H, W, C, lddy, dyoff, dx.data_ptr(), act_f32(dy, "upsample2x_bwd"),
                             cur_stream()),
        "upsample2x_bwd");
}

// entries: int64 tensor [n][16] on the host: src_ptr, dst_ptr, d0..d3, v0..v3, s0..s3, start
// f32: the destinations are fp32 compute copies (fp32 precision path), else bf16
void cast_weights(const at::Tensor& entries_dev, const at::Tensor& block_map_dev, bool f32) {
  check(dlmpi_cast_weights(reinterpret_cast<const CastEntry*>(entries_dev.data_ptr()), block_map_dev.data_ptr(),
                           (int)(block_map_dev.numel() / 4), f32 ? 1 : 0, cur_stream()),
        "cast_weights");
}

// --------------------------------- losses / eval -------------------------------------------
void softmax_ce_fwd(const at::Tensor& logits, int ldl, const at::Tensor& labels, int N, int K, at::Tensor loss_rows,
                    at::Tensor lse, at::Tensor loss) {
  check(dlmpi_softmax_ce_fwd(ptr<float>(logits), ldl, ptr<int64_t>(labels), N, K, ptr<float>(loss_rows),
                             ptr<float>(lse), cur_stream()),
        "softmax_ce_fwd");
  check(dlmpi_sum_f32(ptr<float>(loss_rows), N, ptr<float>(loss), 1.f / (float)N, cur_stream()), "sum");
}
void softmax_ce_bwd(const at::Tensor& logits, int ldl, const at::Tensor& labels, const at::Tensor& lse, int N, int K,
                    int ldd, const c10::optional<at::Tensor>& go, double scale, at::Tensor dlogits) {
  check(dlmpi_softmax_ce_bwd(ptr<float>(logits), ldl, ptr<int64_t>(labels), ptr<float>(lse), N, K, ldd,
                             optr<float>(go), (float)scale, ptr<float>(dlogits), cur_stream()),
        "softmax_ce_bwd");
}
void bce_fwd(const at::Tensor& logits, int ldl, const at::Tensor& target, int64_t M, at::Tensor loss) {
  int nblk = (int)std::min<int64_t>(1024, std::max<int64_t>(1, (M + 4095) / 4096));
  at::Tensor partial = at::empty({nblk}, logits.options().dtype(at::kFloat));
  check(dlmpi_bce_fwd(ptr<float>(logits), ldl, ptr<float>(target), M, ptr<float>(partial), nblk, cur_stream()),
        "bce_fwd");
  check(dlmpi_sum_f32(ptr<float>(partial), nblk, ptr<float>(loss), 1.f / (float)M, cur_stream()), "sum");
}
void bce_bwd(const at::Tensor& logits, int ldl, const at::Tensor& target, int64_t M,
             const c10::optional<at::Tensor>& go, double scale, at::Tensor dlogits) {
  check(dlmpi_bce_bwd(ptr<float>(logits), ldl, ptr<float>(target), M, optr<float>(go), (float)scale,
                      ptr<float>(dlogits), cur_stream()),
        "bce_bwd");
}
void argmax_correct(const at::Tensor& logits, int ldl, const at::Tensor& labels, int N, int K, at::Tensor correct) {
  check(dlmpi_argmax_correct(ptr<float>(logits), ldl, ptr<int64_t>(labels), N, K, ptr<int>(correct), cur_stream()),
        "argmax_correct");
}
void dice(const at::Tensor& logits, int ldl, const at::Tensor& target, int N, int64_t HW, at::Tensor out) {
  check(dlmpi_dice(ptr<float>(logits), ldl, ptr<float>(target), N, HW, ptr<float>(out), cur_stream()), "dice");
}

// --------------------------------- optimizers ----------------------------------------------
void sgd_step(at::Tensor p, const at::Tensor& g, at::Tensor m, double lr, double momentum, double dampening,
              double wd, bool nesterov, bool first, const c10::optional<at::Tensor>& skip_flag) {
  check(dlmpi_sgd(ptr<float>(p), ptr<float>(g), ptr<float>(m), p.numel(), (float)lr, (float)momentum,
                  (float)dampening, (float)wd, nesterov ? 1 : 0, first ? 1 : 0, optr<float>(skip_flag), cur_stream()),
        "sgd");
}
void adam_step(at::Tensor p, at::Tensor g, at::Tensor m, at::Tensor v, double lr, double b1, double b2,
               double eps, double wd, bool adamw, double bc1, double bc2, const c10::optional<at::Tensor>& clip,
               const c10::optional<at::Tensor>& tstep, bool clip_writeback) {
  check(dlmpi_adam(ptr<float>(p), ptr<float>(g), ptr<float>(m), ptr<float>(v), p.numel(), (float)lr, (float)b1,
                   (float)b2, (float)eps, (float)wd, adamw ? 1 : 0, (float)bc1, (float)bc2, optr<float>(clip),
                   optr<float>(tstep), clip_writeback ? 1 : 0, cur_stream()),   // tstep advanced in place unless skipped
        "adam");
}
// total L2 norm of a flat fp32 buffer -> norm_out[0]; coef_out = {min(1, max_norm/(norm+1e-6)), nonfinite}
void grad_norm(const at::Tensor& g, double max_norm, at::Tensor norm_out, at::Tensor coef_out) {
  const int nblk = 1024;
  at::Tensor partial = at::empty({nblk}, g.options().dtype(at::kFloat));
  check(dlmpi_sumsq(ptr<float>(g), g.numel(), ptr<float>(partial), nblk, cur_stream()), "sumsq");
  if (coef_out.numel() < 2) throw std::runtime_error("grad_norm: coef_out needs 2 (or 4) floats");
  check(dlmpi_clip_coef(ptr<float>(partial), nblk, (float)max_norm, ptr<float>(norm_out), ptr<float>(coef_out),
                        (int)std::min<int64_t>(4, coef_out.numel()), cur_stream()),
        "clip_coef");
}
void scale_(at::Tensor x, const at::Tensor& coef) {
  check(dlmpi_scale_f32(ptr<float>(x), x.numel(), ptr<float>(coef), cur_stream()), "scale");
}

// --------------------------------- utilities -----------------------------------------------
void fill_(at::Tensor t, double v) {
  if (t.scalar_type() != at::kFloat || !t.is_contiguous()) throw std::runtime_error("fill_: contiguous fp32 tensor");
  check(dlmpi_fill_f32(ptr<float>(t), t.numel(), (float)v, cur_stream()), "fill");
}
// t: int64 [blocks][4] on the device (bench.py clock stamps)
void clock_stamp(at::Tensor t) {
  if (t.scalar_type() != at::kLong || !t.is_contiguous() || t.dim() != 2 || t.size(1) != 4)
    throw std::runtime_error("clock_stamp: contiguous int64 [blocks][4]");
  check(dlmpi_clock_stamp(reinterpret_cast<unsigned long long*>(t.data_ptr<int64_t>()), (int)t.size(0), cur_stream()),
        "clock_stamp");
}
void add_i64_(at::Tensor t, int64_t v) {
  if (t.scalar_type() != at::kLong || !t.is_contiguous()) throw std::runtime_error("add_i64_: contiguous int64 tensor");
  check(dlmpi_add_i64(ptr<int64_t>(t), t.numel(), v, cur_stream()), "add_i64");
}
// dst.view(-1)[i] (+)= src.view(-1)[idx[i]]  (idx < 0: 0), every i < idx.numel()
void gather_(at::Tensor dst, const at::Tensor& src, const at::Tensor& idx, bool accumulate) {
  if (dst.scalar_type() != src.scalar_type() || !dst.is_contiguous() || !src.is_contiguous() ||
      idx.scalar_type() != at::kLong || !idx.is_contiguous() || idx.numel() > dst.numel())
    throw std::runtime_error("gather_: contiguous dst/src of one dtype, int64 idx no longer than dst");
  check(dlmpi_gather(dst.data_ptr(), src.data_ptr(), ptr<int64_t>(idx), idx.numel(), (int)dst.element_size(),
                     accumulate ? 1 : 0, cur_stream()),
        "gather");
}

// --------------------------------- device-resident input pipeline ---------------------------
void image_batch(const at::Tensor& data, const at::Tensor& labels, const at::Tensor& idx, int H, int W, int C,
                 int pad, bool augment, int64_t seed, int64_t epoch, std::vector<double> mean, std::vector<double> sd,
                 at::Tensor out, const c10::optional<at::Tensor>& out_labels) {
  require_gpu(data, "data");
  if (mean.size() != (size_t)C || sd.size() != (size_t)C) throw std::runtime_error("image_batch: mean/std per channel");
  if (data.scalar_type() != at::kByte || idx.scalar_type() != at::kLong || out.scalar_type() != at::kFloat)
    throw std::runtime_error("image_batch: uint8 data, int64 indices, fp32 output");
  float m3[3] = {0.f, 0.f, 0.f}, s3[3] = {1.f, 1.f, 1.f};
  for (int c = 0; c < C; ++c) { m3[c] = (float)mean[c]; s3[c] = (float)sd[c]; }
  const int B = (int)idx.numel();
  if (out.numel() != (int64_t)B * C * H * W) throw std::runtime_error("image_batch: output size");
  check(dlmpi_image_batch(ptr<uint8_t>(data), ptr<int64_t>(labels), ptr<int64_t>(idx), B, H, W, C, pad, augment ? 1 : 0,
                          (uint32_t)seed, (uint32_t)epoch, m3, s3, ptr<float>(out), optr<int64_t>(out_labels),
                          cur_stream()),
        "image_batch");
}

void register_ops(pybind11::module& m) {
  namespace py = pybind11;
  m.def("conv2d_fwd", &conv2d_fwd);
  m.def("conv2d_fwd_pro", &conv2d_fwd_pro);
  m.def("conv2d_fwd_bn", &conv2d_fwd_bn);
  m.def("conv2d_fwd_mtiles", &conv2d_fwd_mtiles);
  m.def("conv2d_fwd_mtiles_pro", &conv2d_fwd_mtiles_pro);
  m.def("conv2d_fwd_bnbwd", &conv2d_fwd_bnbwd);
  m.def("conv2d_dgrad", &conv2d_dgrad);
  m.def("conv2d_dgrad_pro", &conv2d_dgrad_pro);
  m.def("convT2x2_fwd", &convT2x2_fwd);
  m.def("conv2d_wgrad", &conv2d_wgrad);
  m.def("conv2d_wgrad_pro", &conv2d_wgrad_pro);
  m.def("bn_finalize", &bn_finalize);
  m.def("set_aux_stream", [](int64_t h, int role) {
    check(dlmpi_set_aux_stream(reinterpret_cast<hipStream_t>(h), role), "set_aux_stream");
  });
  // bounded spin kernel on the current stream (tests: delays a collective to expose missing fences)
  m.def("delay_ms", [](double ms) { check(dlmpi_delay(ms, cur_stream()), "delay_ms"); });
  // reads and resets HIP's per-thread sticky error (a failed hipGraph capture leaves
  // hipErrorStreamCaptureInvalidated behind, which the next checked launch would report)
  m.def("clear_hip_error", []() { return (int)hipGetLastError(); });
  // raw HIP streams (not torch pool streams: one that a failed capture leaves in capture mode is
  // simply abandoned, never handed out again)
  m.def("create_stream", []() {
    hipStream_t s = nullptr;
    check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreateWithFlags");
    return reinterpret_cast<int64_t>(s);
  });
  m.def("stream_capturing", [](int64_t h) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    const hipError_t e = hipStreamIsCapturing(reinterpret_cast<hipStream_t>(h), &st);
    (void)hipGetLastError();
    return e != hipSuccess || st != hipStreamCaptureStatusNone;
  });
  m.def("reduce_blocks", &reduce_blocks);
  m.def("bn_stats", &bn_stats);
  m.def("bn_apply", &bn_apply);
  m.def("bn_bwd_reduce", &bn_bwd_reduce);
  m.def("bn_bwd_finalize", &bn_bwd_finalize);
  m.def("bn_bwd_finalize_fused", &bn_bwd_finalize_fused);
  m.def("bn_bwd_apply", &bn_bwd_apply);
  m.def("dual_dgrad_weights", &dual_dgrad_weights);
  m.def("channel_sum", &channel_sum);
  m.def("maxpool_fwd", &maxpool_fwd, py::arg("x"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"),
        py::arg("ldx"), py::arg("xoff"), py::arg("k"), py::arg("stride"), py::arg("pad"), py::arg("y"), py::arg("idx"),
        py::arg("OH"), py::arg("OW"), py::arg("scale"), py::arg("shift"), py::arg("ys") = py::none(),
        py::arg("ldys") = 0, py::arg("ysoff") = 0);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("maxpool_bwd_bn", &maxpool_bwd_bn);
  m.def("outer_dgrad_bn", &outer_dgrad_bn);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("nchw_to_nhwc", &nchw_to_nhwc);
  m.def("s2d_nchw", &s2d_nchw);
  m.def("image_batch", &image_batch);
  m.def("upsample2x_fwd", &upsample2x_fwd);
  m.def("upsample2x_bwd", &upsample2x_bwd);
  m.def("cast_weights", &cast_weights);
  m.def("softmax_ce_fwd", &softmax_ce_fwd);
  m.def("softmax_ce_bwd", &softmax_ce_bwd);
  m.def("bce_fwd", &bce_fwd);
  m.def("bce_bwd", &bce_bwd);
  m.def("argmax_correct", &argmax_correct);
  m.def("dice", &dice);
  m.def("sgd_step", &sgd_step);
  m.def("adam_step", &adam_step);
  m.def("grad_norm", &grad_norm);
  m.def("scale_", &scale_);
  m.def("fill_", &fill_);
  m.def("set_conv_stream", [](int mode) { dlmpi_set_conv_stream(mode); });
  m.def("conv_stream_last", []() { return g_stream_ran; });
  m.def("set_dgrad_stream", [](int mode) { dlmpi_set_dgrad_stream(mode); });
  m.def("dgrad_stream_last", []() { return g_dgrad_stream_ran; });
  m.def("set_conv_autotune", [](int mode) { g_autotune_override = mode; });
  m.def("set_wgrad3", [](int mode) { g_wgrad3_override = mode; });
  m.def("set_wgrad3_blocks", [](int n) { g_wgrad3_blocks = n; });
  m.def("set_head1x1", [](int v) { g_head_on = v; });
  m.def("head1x1_on", []() { return g_head_on; });
  m.def("conv1x1_head_affine", &conv1x1_head_affine);
  m.def("set_conv_c8", [](int v) { g_c8_on = v; });
  m.def("set_conv_c16", [](int v) { g_c16_on = v; });
  m.def("set_conv3_pro", [](int v) { g_c3pro_on = v; });
  m.def("conv3_pro_ok", &conv3_pro_ok);
  m.def("conv3x3_fwd_bn_apply", &conv3x3_fwd_bn_apply);
  m.def("conv_c16_last", []() { return g_c16_ran; });
  m.def("set_convT_stream", [](int v) { g_convT_stream = v; });
  m.def("convT_stream_last", []() { return g_convT_stream_ran; });
  m.def("conv_c8_last", []() { return g_c8_ran; });
  m.def("head1x1_last", []() { return g_head_ran; });
  m.def("set_wgrad_defer", [](bool on) {
    if (!on) wgrad_flush();
    g_wgrad_defer = on;
  });
  m.def("wgrad_flush", &wgrad_flush);
  m.def("wgrad_discard", &wgrad_discard);
  m.def("clock_stamp", &clock_stamp);
  m.def("set_wgrad_batch", [](int n) { g_wgrad_batch = n > 0 && n <= dlmpi::kWgradBatch ? n : dlmpi::kWgradBatch; });
  m.def("set_defer_direct", [](int on) { g_defer_direct = on != 0; });
  m.def("set_wgrad_bypass", [](bool on) { g_wgrad_bypass = on; });
  m.def("wgrad_pending", []() { return (int)g_pending.size(); });
  m.def("wgrad_reduce_launches", []() { return g_reduce_launches; });
  m.def("set_conv_halo", [](int mode) { g_halo_override = mode; });
  m.def("set_halo_first", [](int on) { g_halo_first = on; });
  m.def("set_halo_pipe", [](int on) { dlmpi_set_halo_pipe(on); });
  m.def("set_wgrad_fast", [](int on) { dlmpi_set_wgrad_fast(on); });
  m.def("set_wgrad_blocks", [](int n) { g_wgrad_blocks = n; });
  m.def("set_conv_splitk", [](int n) { g_splitk_override = n; });
  m.def("set_conv_pipe_dgrad", [](int mode) { g_pipe_dgrad_override = mode; });
  m.def("set_conv_pipe", [](int mode) { g_pipe_override = mode; });
  m.def("set_conv_apply", [](int mode) { g_apply_override = mode; });
  m.def("set_conv3_stream", [](int mode) { dlmpi_set_conv3_stream(mode); });
  m.def("conv3_stream_last", []() { return g_conv3_ran; });
  m.def("set_dgs_blocks", [](int n) { dlmpi_set_dgs_blocks(n); });
  m.def("dgs_blocks", []() { return dlmpi_dgs_blocks(); });
  m.def("conv_halo_last", []() { return g_halo_ran; });
  m.def("conv2d_fwd_bn_apply", &conv2d_fwd_bn_apply);
  m.def("wgrad3_last", []() { return g_wgrad3_ran; });
  m.def("clear_conv_plans", []() { g_conv_plans.clear(); });
  m.def("add_i64_", &add_i64_);
  m.def("gather_", &gather_);
  m.attr("CAST_ENTRY_BYTES") = (int)sizeof(CastEntry);
}

}  // namespace dlmpi_ext
