// Host-visible interface of the gfx950 kernel library (pure HIP, no torch dependency).
// Included by the .hip kernel files and by the torch binding (compiled with g++).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace dlmpi {

// Unsigned fast division by a runtime constant, valid for n < 2^31:
// q = (mulhi(n, m) + n) >> l with l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1.
struct FastDiv {
  uint32_t d, mul, shr;
};
inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  f.mul = (uint32_t)((((1ull << 32) * ((1ull << l) - d)) / d) + 1);
  f.shr = l;
  return f;
}

// ---------------------------------------------------------------------------------------------
// Implicit-GEMM convolution on MFMA (forward, data-gradient, transposed-conv forward, linear).
//
// GEMM rows   m = (n, p, q) over an output grid P x Q of one "phase";
// GEMM cols   k = output channel (Kout);
// reduction   over taps t = (tr, ts) in a Tr x Ts grid and C input channels.
// For tap t the A row reads input pixel  ih = p*sa + dh0 + tr*dhs,  iw = q*sa + dw0 + ts*dws
// and the B row reads weight tap index   (wr0 + tr*wrs)*S + (ws0 + ts*wss)  of a [Kout][R][S][C]
// weight.  The result goes to output pixel (p*so + oh0, q*so + ow0).
// A forward conv is one phase (sa = stride, dh0 = -pad); a strided data-gradient or a
// transposed conv is stride^2 phases (sub-pixel decomposition), selected by blockIdx.z.
// ---------------------------------------------------------------------------------------------
// Per-channel BatchNorm finalize arguments (bn.hip colsum kernels and the in-launch finalize of
// the conv epilogue, bnfin.h).
struct FinArgs {
  int mode;   // 0: forward statistics -> scale/shift (+ running stats); 1: backward coefficients
  double count;
  const float* gamma;
  const float* beta;
  float* running_mean;
  float* running_var;
  float momentum, eps;
  float* scale;
  float* shift;
  float* save_mean;
  float* save_invstd;
  const float* mean;     // backward
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* coef;
  int raw_z;
};

// Streaming 1x1 forward (conv1x1_stream.hip): y[m][yoff + n] = sum_c x[row(m)][xoff + c] w[n][c]
// (+ bias[n]) for m < M, bf16; stats (or null): [G][2][Kout] partial sums of the stored values, one
// row per block of an N-tile.  row(m) = m (stride 1) or, with s2, the input pixel (n, 2p, 2q) of
// output pixel m = (n, p, q) of a P x Q grid over an H x W input (the stride-2 projection).
struct Stream1x1Args {
  const uint16_t* x;
  int ldx, xoff;
  const uint16_t* w;               // [Kout][C]
  uint16_t* y;
  int ldy, yoff;
  int y_bytes;                     // buffer-descriptor range of y (rows past M are dropped)
  int M, C, Kout;
  const float* bias;
  float* stats;
  int G, ntiles, mtiles;
  int s2, H, W;                    // stride-2 gather (s2 = 1): input grid
  FastDiv fdPQ, fdQ;               // output grid P x Q
  int up2;                         // 1: ConvTranspose2d(2, 2): Kout = 4 Cup rows (i, j, co), w [Cup][2][2][C],
  int Cup;                         //    output pixel (2h + i, 2w + j); fdPQ / fdQ = the input grid H W / W
};

// Streaming 1x1 / stride-1 data gradient with the fused BN-backward epilogue (conv1x1_dgrad_stream.hip)
struct DgradStreamArgs {
  const uint16_t* x;               // GEMM A operand [M][ldx] (K channels at xoff): dy, or [dy | z]
  int ldx, xoff;
  const uint16_t* w;               // [Kout][K]
  uint16_t* y;                     // dx [M][ldy] (Kout channels at yoff)
  int ldy, yoff;
  int y_bytes;
  int M, K, Kout;
  const float* bias;               // fp32 [Kout] or null (dual: W . k3)
  const uint16_t* res;             // residual gradient added before the mask, or null
  int ldres, resoff;
  const uint16_t* z;               // BN input of the consumer (statistics, z-mask), or null
  int ldz, zoff;
  const uint16_t* z2;              // a second BN input consuming the same gradient (ResNet downsample)
  int ldz2, z2off;
  const uint8_t* mbits;            // [M][Kout / 8] ReLU mask bits (mask mode 1)
  const float* mscale;             // mask mode 2: keep where z * mscale + mshift > 0
  const float* mshift;
  float* stats;                    // [G][2|3][Kout] {sum dx, sum dx * z [, sum dx * z2]} per block
  int G, ntiles, mtiles;
};

struct ConvPhase {
  int P, Q;
  int Tr, Ts;
  int dh0, dhs, dw0, dws;
  int wr0, wrs, ws0, wss;
  int oh0, ow0;
  int mtiles;   // ceil(N*P*Q / BM)
  int ksteps;   // ceil(Tr*Ts*C / 64)
  int tile_base;  // first stats row of this phase (phases' tiles are numbered consecutively)
  FastDiv fdPQ, fdQ, fdTs;
};

struct ConvArgs {
  const void* x;                   // bf16 (uint16_t) or, with f32 = 1, float elements
  int H, W, C, ldx, xoff;          // input NHWC, pixel stride ldx, channel offset xoff
  const void* w;
  int ldw, S;                      // weight row stride (= R*S*C), S of the weight tap grid
  void* y;
  int OH, OW, ldy, yoff;           // output NHWC geometry
  int so, sa;                      // output / input coordinate multipliers
  int out_f32;                     // 1: fp32 output, 0: bf16 output
  int Nimg, Kout;
  int kvalid;                      // output channels actually stored (<= Kout)
  int vec_store;                   // 1: 16-byte stores legal (ldy, yoff multiples of 8 and kvalid == Kout)
  const float* bias;               // [Kout] or null
  const void* res;             // residual added in the epilogue (same pixel grid as y) or null
  int ldres, resoff;
  const float* scale;              // per-channel affine after bias (folded eval BN) or null
  const float* shift;
  int relu;
  float* stats;                    // BN partial sums [tiles][nstat][Kout] of the (bf16-rounded) output, or null
  // Backward fusion (the GEMM produces the gradient dy of a BatchNorm+ReLU output y):
  //   v := v * [mask > 0] (ReLU derivative) before the store, and the stats become
  //   {sum v, sum v*z [, sum v*z2]} with z (z2) the BN input(s) that consume this gradient.
  const void* mask;            // ReLU output y (mask = y > 0), or null with mscale set:
  int ldmask, maskoff;
  const float* mscale;             //   mask = z * mscale + mshift > 0 (BN+ReLU without residual:
  const float* mshift;             //   recomputed from z, which the stats read anyway)
  const uint8_t* mbits;            //   or mask bits written by the forward BN-apply ([pix][Kout/8])
  const void* z;
  int ldz, zoff;
  const void* z2;
  int ldz2, z2off;
  int nstat;                       // 2 (fwd: sum v, sum v^2; bwd: sum v, sum v*z) or 3 (bwd with z2)
  int ntiles;
  int nphase;
  int splitk;                      // > 1: K split over blockIdx.y, last-arriver combine (set by the launcher)
  int splitk_req;                  // 0: the launcher plans the split; >= 1: use exactly this (autotuner)
  float* sk_slab;                  // [tile][slice][TM*TN][threads] f32x4 fragment slabs
  int* sk_tk;                      // [tile] self-resetting arrival tickets
  int cstep, tstep;                // K-iteration: c += cstep, t += tstep per 64-wide step
  // Operand prologue (single-stage kernel, regular channel counts), pro 3 (1x1 / stride 1
  // consumers): every staged A piece is rewritten in LDS before the MFMAs as A := bf16(relu(A *
  // pscale[c] + pshift[c] + R)), R = Z (the residual, staged like A) or Z * prscale[c] + prshift[c]
  // (a BN-output residual); output tile column 0 also stores it to py and its ReLU mask bits to
  // pmbits [pixels][C/8] (the producer block's BN-apply, fused); pro 0: none
  int pro;
  int f32;                         // 1: activations / weights are fp32 (the fp32 precision path)
  const float* pscale;
  const float* pshift;
  const void* pz;
  int ldpz, pzoff;
  const float* prscale;
  const float* prshift;
  uint16_t* py;
  int ldpy, pyoff;
  uint8_t* pmbits;
  // 2-D halo tiles (conv_igemm.hip HALO; 3x3 / stride 1 / pad 1, one phase): M-tile mt = (n, ti, tj)
  // of the N x tiles_h x tiles_w grid covers output pixels [ti th, +th) x [tj tw, +tw)
  int halo;
  int th, tw, tiles_h, tiles_w;
  FastDiv fd_tw, fd_tilesw, fd_thw;
  ConvPhase ph[4];
};

// ---------------------------------------------------------------------------------------------
// Weight gradient:  dW[ko][t][c] = sum_pix dY[pix][ko] * X[gather(pix, t)][c]   (split over pix)
// ---------------------------------------------------------------------------------------------
struct WgradArgs {
  const void* dy;                  // bf16 (uint16_t) or, with f32 = 1, float elements
  int ldy, dyoff, Ko;
  const void* x;
  int H, W, C, ldx, xoff;
  int Nimg, P, Q, S, stride_h, stride_w, pad_h, pad_w;
  int TC;                          // R*S*C
  int npix, pix_per_split;
  int mtiles, ntiles, splits;
  int direct;                      // 1: 1x1 / stride 1 / pad 0 on the same grid (no gather decode)
  FastDiv fdPQ, fdQ, fdC, fdS;
  float* ws;                       // [splits][Ko][TC] fp32 partials (reduced by dlmpi_wgrad_reduce)
  // Operand prologues (conv_igemm's pro modes, applied in LDS to in-range pieces only):
  //   dy side (A): pro_a 2 -> dz = pcoef[k] * dy + pcoef[Ko + k] * Z + pcoef[2 Ko + k]
  //   x side  (B): pro_b 1 -> x := relu(x * pscale[c] + pshift[c])
  int pro_a, pro_b;
  int f32;                         // 1: fp32 operands (conv_wgrad_f32_kernel, 64 x 64 tiles)
  const float* pcoef;
  const uint16_t* pz;
  int ldpz, pzoff;
  const float* pscale;
  const float* pshift;
  int fast;                        // set by dlmpi_conv_wgrad: scalar-base DMA staging allowed (A/B knob)
};

// Streaming 3x3 / stride-1 / pad-1 convolution, 64 -> 64 channels (conv3x3_stream.hip): persistent
// blocks over th x tw output tiles with all 9 taps' weights resident.  Forward (w [64][3][3][64],
// flip 0) or stride-1 data gradient (w = wT [C][3][3][K], flip 1); mode 0: + bias, statistics
// {sum y, sum y^2}; 1: plain; 2: dgrad into a BN + ReLU output (mask z * mscale + mshift > 0,
// statistics {sum dx, sum dx * z}); stats [G][2][64].
struct Conv3StreamArgs {
  const uint16_t* x;
  int ldx, xoff;
  const uint16_t* w;
  int ldw, flip;
  uint16_t* y;
  int ldy, yoff;
  int N, H, W;
  int th, tw, tiles_h, tiles_w, ntiles, G;
  const float* bias;
  const uint16_t* z;
  int ldz, zoff;
  const float* mscale;
  const float* mshift;
  float* stats;
  // forward with the producer's BN-apply + ReLU fused (conv3x3_stream_kernel PRO): x is the producer
  // BN's input z; the kernel stages relu(z * psc + psh) and stores it (each pixel once) to py
  const float* psc;
  const float* psh;
  uint16_t* py;
  int ldpy, pyoff;
};

// 3x3 / stride-1 / pad-1 weight gradient by 8 x 8 output-pixel tiles (conv_wgrad3.hip): split z
// reduces pixel tiles [z * tiles_per_split, ...) of the N x tiles_h x tiles_w grid into
// ws[z][Ko][9 * C] (tap-major columns, the general path's workspace layout)
// One deferred split reduction of a weight gradient (dlmpi_wgrad_reduce_batch): the same sums in
// the same order as dlmpi_wgrad_reduce(ws, splits, Ko, T, Cpad, Creal, Ko_real, out, ws2, ...).
struct WgradReduceEntry {
  const float* ws;                 // [splits][Ko][T][Cpad] partials
  float* ws2;                      // [G][Ko][T][Cpad] group sums (G > 0)
  float* out;                      // [Ko_real][T][Creal], accumulated
  int64_t total;                   // Ko * T * Cpad
  int splits, G, Ko_real, T, Cpad, Creal;
  int block1;                      // first block of this entry in the stage-1 grid (G > 0)
  int block2;                      // first block of this entry in the stage-2 grid
};
constexpr int kWgradBatch = 16;
struct WgradReduceBatch {
  int n;
  WgradReduceEntry e[kWgradBatch];
};

struct Wgrad3Args {
  const void* dy;
  int ldy, dyoff, Ko;
  const void* x;
  int ldx, xoff, C;
  int H, W;                        // input = output grid (stride 1, pad 1)
  int tiles_h, tiles_w, ntiles_pix, tiles_per_split;
  int mtiles, ntiles, splits;      // Ko / KT, C / CT, pixel splits
  float* ws;
};

}  // namespace dlmpi

extern "C" {
// conv / gemm
void dlmpi_set_wgrad_fast(int on);  // conv_wgrad_kernel scalar-base DMA staging (A/B)
void dlmpi_set_halo_pipe(int on);   // 256 x 128 halo tiles on the weight-double-buffered kernel (A/B)
hipError_t dlmpi_conv_igemm(const dlmpi::ConvArgs* a, int bm, int bn, hipStream_t s);
// pipe = 1: the pipelined 8-wave kernel (tiles 256x256, 256x128, 128x256, 256x64, 512x64; bf16,
// C % 64 == 0, no prologue / halo / split); pipe = 0: dlmpi_conv_igemm
hipError_t dlmpi_conv_igemm_ex(const dlmpi::ConvArgs* a, int bm, int bn, int pipe, hipStream_t s);
// pro-3 (fused producer BN-apply) 1x1 / stride-1 launches with one 64 / 128 / 256-channel output
// column: the register-staged kernel (conv_igemm.hip conv1x1_apply_kernel), 128-row tiles
int dlmpi_conv1x1_apply_ok(int C, int K);
hipError_t dlmpi_conv1x1_apply(const dlmpi::ConvArgs* a, int bm, hipStream_t s);
hipError_t dlmpi_conv_wgrad(const dlmpi::WgradArgs* a, int bm, int bn, hipStream_t s);   // bn: 128 | 256
// 1 if dlmpi_conv_wgrad has the operand-prologue combination (pro_a 2 / pro_b 1) for this gradient
int dlmpi_wgrad_pro_ok(int direct, int pro_a, int pro_b);
// sum of split partials -> grad (accumulated), with channel un-padding and row limit
hipError_t dlmpi_wgrad_reduce(const float* ws, int splits, int Ko, int T, int Cpad, int Creal,
                              int Ko_real, float* out, float* ws2, int ws2_floats, hipStream_t s);
int dlmpi_wgrad_reduce_groups(int splits, int64_t total);
// up to kWgradBatch deferred reductions in two launches (stage 1 only if an entry has G > 0; G and the
// block offsets are filled in here)
hipError_t dlmpi_wgrad_reduce_batch(dlmpi::WgradReduceBatch* b, hipStream_t s);
// 3x3 spatial-tile weight gradient: tile plan (KT x CT; 0 if the channel counts do not fit) + launch
int dlmpi_wgrad3_plan(int Ko, int C, int* kt, int* ct);
hipError_t dlmpi_wgrad3x3(const dlmpi::Wgrad3Args* a, int kt, int ct, hipStream_t s);
int dlmpi_head1x1_ok(int C, int kv);
int dlmpi_conv3x3_c8_blocks(int64_t pixels);
int dlmpi_conv4x4_c16_blocks(int64_t pixels);
hipError_t dlmpi_conv4x4_c16(const void* x, int ldx, int xoff, int N, int U, int V, const void* w, const float* bias,
                             void* y, int ldy, int yoff, float* stats, int G, hipStream_t s);
hipError_t dlmpi_conv3x3_c8(const void* x, int ldx, int xoff, int N, int H, int W, const void* w, const float* bias,
                            void* y, int ldy, int yoff, float* stats, int G, hipStream_t s);
hipError_t dlmpi_head1x1(const void* x, int ldx, int xoff, int64_t M, int C, const void* w, int ldw,
                         const float* bias, void* y, int ldy, int yoff, int kv, int y_f32, const float* psc,
                         const float* psh, hipStream_t s);
// streaming 64 -> 64 3x3 conv: plan (tile th x tw, G blocks; 0 if it does not apply) + launch
int dlmpi_conv3_stream_plan(int N, int H, int W, int C, int K, int blocks, int* th, int* tw, int* G);
hipError_t dlmpi_conv3x3_stream(const dlmpi::Conv3StreamArgs* a, int mode, hipStream_t s);
void dlmpi_set_conv3_stream(int mode);

// batch norm
hipError_t dlmpi_bn_finalize(const float* partial, int ntiles, int C, double count, const float* gamma,
                             const float* beta, float* running_mean, float* running_var, float momentum,
                             float eps, float* scale, float* shift, float* save_mean, float* save_invstd,
                             double* ws, hipStream_t s);
int dlmpi_colsum_ws_doubles(int T, int C);
// register an auxiliary stream (role 1..3) of the current device: own last-arriver ticket array
hipError_t dlmpi_set_aux_stream(hipStream_t s, int role);
// Activation-typed launchers below take `const void*` / `void*` activations and `int f32`: 1 = fp32
// storage (the fp32 precision path), 0 = bf16 (uint16_t).
hipError_t dlmpi_bn_stats(const void* x, int64_t M, int C, int ldx, int xoff, float* partial, int nblk, int f32,
                          hipStream_t s);
// mbits (optional): [M][C/8] bytes, bit e of byte (row, g) = y[row][8g + e] > 0 (ReLU mask for backward)
hipError_t dlmpi_bn_apply(const void* x, int ldx, int xoff, int64_t M, int C, const float* scale, const float* shift,
                          const void* res, int ldres, int resoff, int relu, void* y, int ldy, int yoff, uint8_t* mbits,
                          int f32, hipStream_t s);
// as dlmpi_bn_apply; the residual is a BN output applied on the fly: res * rscale + rshift
hipError_t dlmpi_bn_apply2(const void* x, int ldx, int xoff, int64_t M, int C, const float* scale, const float* shift,
                           const void* res, int ldres, int resoff, const float* rscale, const float* rshift, int relu,
                           void* y, int ldy, int yoff, uint8_t* mbits, int f32, hipStream_t s);
hipError_t dlmpi_bn_bwd_reduce(const void* dy, int lddy, int dyoff, const void* ymask, int ldym, int ymoff,
                               const void* x, int ldx, int xoff, int64_t M, int C, const float* mean,
                               const float* invstd, float* partial, int nblk, int f32, hipStream_t s);
hipError_t dlmpi_bn_bwd_finalize(const float* partial, int nblk, int C, double count, const float* gamma,
                                 const float* mean, const float* invstd, float* dgamma, float* dbeta,
                                 float* coef, double* ws, hipStream_t s);
// partials [nblk][ns][C]: rows 0 (sum dyr) and k2 (sum dyr*xhat, or sum dyr*z when raw_z)
hipError_t dlmpi_bn_bwd_finalize_ex(const float* partial, int nblk, int ns, int k2, int raw_z, int C, double count,
                                    const float* gamma, const float* mean, const float* invstd, float* dgamma,
                                    float* dbeta, float* coef, double* ws, hipStream_t s);
hipError_t dlmpi_bn_bwd_apply(const void* dy, int lddy, int dyoff, const void* ymask, int ldym, int ymoff,
                              const void* x, int ldx, int xoff, int64_t M, int C, const float* coef, void* dx,
                              void* dyr_out, int f32, hipStream_t s);
// [dy | z] weights of the dual 1x1 data gradient: w2 [C][2K] = {W*k1, W*k2}, b [C] = W . k3 (coef [3][K])
hipError_t dlmpi_dual_dgrad_weights(const void* w, int C, int K, const float* coef, void* w2, float* b, int f32,
                                    hipStream_t s);
hipError_t dlmpi_channel_sum(const void* x, int64_t M, int C, int ldx, int xoff, float* out_acc, float* partial,
                             int nblk, double* ws, int f32, hipStream_t s);
int dlmpi_reduce_blocks(int64_t M, int C);

// pooling / layout
// scale/shift (optional): pool relu(x * scale + shift) (rounded to the storage type), i.e. BN-apply + ReLU fused
hipError_t dlmpi_maxpool_fwd(const void* x, int N, int H, int W, int C, int ldx, int xoff, int k, int stride, int pad,
                             void* y, uint8_t* idx, int OH, int OW, const float* scale, const float* shift, void* ys,
                             int ldys, int ysoff, int f32, hipStream_t s);
hipError_t dlmpi_maxpool_bwd(const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k, int stride,
                             int pad, int OH, int OW, const void* add, int ldadd, int addoff, void* dx, int lddx,
                             int dxoff, int f32, hipStream_t s);
// max-pool backward into the gradient of a BN+ReLU output (mask z*scale+shift > 0), with the BN
// backward partials [nblk][2][C] = {sum dyr, sum dyr*z}; dx/z dense [N*H*W][C]; add (optional): a second
// gradient of the pool input (channel slice of a [N*H*W][ldadd] buffer) summed in before the mask
hipError_t dlmpi_maxpool_bwd_bn(const void* dy, const uint8_t* idx, int N, int H, int W, int C, int k, int stride,
                                int pad, int OH, int OW, const void* z, const float* mscale, const float* mshift,
                                const void* add, int ldadd, int addoff, void* dx, float* partial, int nblk, int f32,
                                hipStream_t s);
// data gradient of a 1x1 conv with one output channel (dx[m,c] = dy[m*lddy] * w[c*ldw]) into the
// gradient of a BN+ReLU output (mask z*scale+shift > 0), BN-backward partials [nblk][2][C]
hipError_t dlmpi_outer_dgrad_bn(const void* dy, int lddy, int64_t M, int C, const void* w, int ldw, const void* z,
                                const float* mscale, const float* mshift, void* dx, float* partial, int nblk, int f32,
                                hipStream_t s);
// per-(device, stream role) split-K workspaces for the conv kernel (bn.hip): an fp32 slab of at least
// `floats` elements and `n` zeroed self-resetting tickets; null if unavailable (e.g. would have to
// grow during a graph capture)
float* dlmpi_splitk_slab(hipStream_t s, size_t floats);
int* dlmpi_splitk_tickets(hipStream_t s, int n);
hipError_t dlmpi_avgpool_fwd(const void* x, int N, int HW, int C, void* y, int f32, hipStream_t s);
hipError_t dlmpi_avgpool_bwd(const void* dy, int N, int HW, int C, void* dx, int f32, hipStream_t s);
hipError_t dlmpi_nchw_to_nhwc(const float* x, int N, int C, int H, int W, int Cpad, void* y, int f32, hipStream_t s);
// 2x2 space-to-depth of the zero-padded image: y [N][U][V][4*CS], slot (vh*2+vw) holds CS channels
hipError_t dlmpi_s2d_nchw(const float* x, int N, int C, int H, int W, int pad, int U, int V, int CS, void* y, int f32,
                          hipStream_t s);
hipError_t dlmpi_upsample2x_fwd(const void* x, int N, int H, int W, int C, int ldx, int xoff, void* y, int ldy,
                                int yoff, int f32, hipStream_t s);
// bilinear x2 (align_corners) backward as a deterministic gather: dx dense [N*H*W][C]
hipError_t dlmpi_upsample2x_bwd(const void* dy, int N, int H, int W, int C, int lddy, int dyoff, void* dx, int f32,
                                hipStream_t s);

// weights: multi-tensor strided 4-D gather + cast fp32 -> bf16 / fp32 (f32 = 1) with zero padding
struct CastEntry {
  const float* src;
  void* dst;
  int d[4];        // destination dims (contiguous)
  int valid[4];    // indices >= valid are zero
  int64_t st[4];   // source strides (elements)
  int64_t start;   // first destination element of this entry in the global enumeration
};
// block_map_dev: int4 per block {entry, slice, slices of that entry, 0}
hipError_t dlmpi_cast_weights(const CastEntry* entries_dev, const void* block_map_dev, int nblocks, int f32,
                              hipStream_t s);

// losses (forward saves what the backward needs; backward reads the upstream grad from device)
hipError_t dlmpi_softmax_ce_fwd(const float* logits, int ldl, const int64_t* labels, int N, int K, float* loss_rows,
                                float* lse, hipStream_t s);
hipError_t dlmpi_softmax_ce_bwd(const float* logits, int ldl, const int64_t* labels, const float* lse, int N, int K,
                                int ldd, const float* go, float scale, float* dlogits, hipStream_t s);
hipError_t dlmpi_bce_fwd(const float* logits, int ldl, const float* target, int64_t M, float* partial, int nblk,
                         hipStream_t s);
hipError_t dlmpi_bce_bwd(const float* logits, int ldl, const float* target, int64_t M, const float* go, float scale,
                         float* dlogits, hipStream_t s);
hipError_t dlmpi_sum_f32(const float* x, int64_t n, float* out, float scale, hipStream_t s);

// eval
hipError_t dlmpi_argmax_correct(const float* logits, int ldl, const int64_t* labels, int N, int K, int* correct,
                                hipStream_t s);
hipError_t dlmpi_dice(const float* logits, int ldl, const float* target, int N, int64_t HW, float* dice,
                      hipStream_t s);

// optimizers on flat fp32 buffers
hipError_t dlmpi_sgd(float* p, const float* g, float* m, int64_t n, float lr, float momentum, float dampening,
                     float wd, int nesterov, int first, const float* skip_flag, hipStream_t s);
hipError_t dlmpi_adam(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1, float b2,
                      float eps, float wd, int adamw, float bc1, float bc2, const float* clip_coef,
                      float* tstep, int wb, hipStream_t s);   // tstep (device step count) overrides bc1/bc2
hipError_t dlmpi_sumsq(const float* x, int64_t n, float* partial, int nblk, hipStream_t s);
hipError_t dlmpi_clip_coef(const float* partial, int nblk, float max_norm, float* norm_out, float* coef_out, int ncoef,
                           hipStream_t s);
hipError_t dlmpi_scale_f32(float* x, int64_t n, const float* coef, hipStream_t s);

// device-resident input pipeline: out[b] = normalize(augment(data[idx[b]])), [B][C][H][W] fp32 (C <= 3)
hipError_t dlmpi_image_batch(const uint8_t* data, const int64_t* labels, const int64_t* idx, int B, int H, int W,
                             int C, int pad, int augment, uint32_t seed, uint32_t epoch, const float* mean3,
                             const float* std3, float* out, int64_t* out_labels, hipStream_t s);

// fault injection: keep stream s busy for `ms` milliseconds (bounded; tests of the watchdog)
hipError_t dlmpi_delay(double ms, hipStream_t s);
// comm-load rehearsal: `channels` workgroups (lds_bytes of LDS each) copy copy_bytes of the bucket
// into scratch and hold their CUs for `us` microseconds (fault.hip)
hipError_t dlmpi_comm_load(const void* bucket, int64_t bytes, void* scratch, int64_t copy_bytes, int channels,
                           int lds_bytes, double us, hipStream_t s);
void dlmpi_set_conv_stream(int mode);
void dlmpi_set_dgrad_stream(int mode);
int dlmpi_stream1x1_plan(int64_t M, int C, int Kout, int stride, int* bm, int* bn, int* G);
hipError_t dlmpi_conv1x1_stream(const dlmpi::Stream1x1Args* a, int bm, int bn, hipStream_t s);
int dlmpi_dgrad_stream_plan(int64_t M, int K, int Kout, int mask_mode, int z2, int has_res, int* bm, int* bn, int* G);
void dlmpi_set_dgs_blocks(int n);
int dlmpi_dgs_blocks();
hipError_t dlmpi_conv1x1_dgrad_stream(const dlmpi::DgradStreamArgs* a, int bm, int bn, int mask_mode, hipStream_t s);

// utilities (util.hip): fp32 fill, int64 add, indexed gather dst[i] (+)= src[idx[i]] (idx < 0: zero;
// esize 2 | 4 bytes, accumulate: fp32 only)
hipError_t dlmpi_fill_f32(float* p, int64_t n, float v, hipStream_t s);
// out [blocks][3] uint64: {XCC id, s_memtime, s_memrealtime} per one-wave block (bench clock stamps)
hipError_t dlmpi_clock_stamp(unsigned long long* out, int blocks, hipStream_t s);
hipError_t dlmpi_add_i64(int64_t* p, int64_t n, int64_t v, hipStream_t s);
hipError_t dlmpi_gather(void* dst, const void* src, const int64_t* idx, int64_t n, int esize, int accumulate,
                        hipStream_t s);

// comm helpers
hipError_t dlmpi_pack(const void* const* srcs, const int64_t* offs, int n, int64_t total_bytes, void* dst,
                      hipStream_t s);
}
