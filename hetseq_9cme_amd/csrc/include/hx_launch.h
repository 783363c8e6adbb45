// Host-callable launchers of the gfx950 kernels.  Pure C++ signatures (raw
// pointers + hipStream_t) so the kernel TUs never include torch headers; the
// torch-facing argument checking lives in csrc/bindings.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// optim.hip
int hx_grad_norm_partials();
void hx_grad_norm_clip(const float* g, int64_t n, double* partial_ws, float* gscale, float* out_norm, float* clipped,
                       float max_norm, hipStream_t s);
// --find-unused device path (optim.hip): table = [nblocks][3] int64 (param, start, end) slices
// of <= hx_adam_mask_chunk() floats, used = all-reduced f64 flags, steps/hp = device state.
int hx_adam_mask_chunk();
void hx_adam_masked(float* p, const float* g, float* m, float* v, uint16_t* shadow, const float* gscale,
                    const int64_t* table, int nblocks, const double* used, int* steps, float* hp, int nparam,
                    double lr, double b1, double b2, float eps, double wd, const double* lr_dev, hipStream_t s);
void hx_adam(float* p, const float* g, float* m, float* v, uint16_t* shadow, const float* gscale, int64_t n, float b1,
             float b2, float eps, float step_size, float wd_lr, const float* hp,
             hipStream_t s);
void hx_adadelta(float* p, const float* g, float* sq, float* acc, const float* gscale, int64_t n, float lr, float rho,
                 float eps, float wd, const float* hp, hipStream_t s);

// layernorm.hip
// amax_part (fp32 only, may be null): max |output| of every row, [rows] (the backward: max |dy|, or
// |dz| without dy) -- the fp16x3 GEMMs' per-row operand scale; colmax (backward, may be null): max
// |dy| (|dz|) of every column, [H] -- the weight gradient's per-column scale.  The backward's
// partial workspace is [nblk][4][H].
int hx_ln_bwd_blocks(int64_t rows);
int hx_ln_fwd_blocks(int64_t rows);
void hx_ln_fwd(int bf16, const void* y, const float* bias, const void* res, const float* gamma, const float* beta,
               void* out, void* zsave, float* mean, float* rstd, int64_t rows, int H, float eps, float keep_prob,
               const uint64_t* seed, uint64_t stream, int drop_after, hipStream_t s, float* amax_part = nullptr,
               uint16_t* pieces = nullptr);   // pieces: fp16 P2 [rows][2H] of out at its row scales
void hx_ln_bwd(int bf16, const void* dout, const void* z, const float* mean, const float* rstd, const float* gamma,
               void* dz, void* dy, float* partial, int nblk, int64_t rows, int H, float keep_prob, const uint64_t* seed,
               uint64_t stream, int drop_after, int want_dbias, float* dgamma, float* dbeta, float* dbias,
               int accumulate, hipStream_t s, float* amax_part = nullptr, float* colmax = nullptr,
               uint16_t* pieces = nullptr);   // pieces: of dy (dz without dy), as hx_ln_fwd
void hx_embed_ln_fwd(int bf16, const int64_t* ids, const int64_t* tt, const float* wte, const float* wpe,
                     const float* wtt, const float* gamma, const float* beta, void* out, void* zsave, float* mean,
                     float* rstd, int64_t rows, int S, int H, float eps, float keep_prob, const uint64_t* seed,
                     uint64_t stream, hipStream_t s, float* amax_part = nullptr, uint16_t* pieces = nullptr);
// token-type embedding gradient for ntypes <= 3: dwtt[t] = sum of dz rows with tt == t (part: a
// [hx_type_grad_blocks(rows)][ntypes][H] fp32 workspace; deterministic block partials + fold)
int hx_type_grad_blocks(int64_t rows);
void hx_type_grad(int bf16, const void* dz, const int64_t* tt, float* part, float* dwtt, int64_t rows, int H, int ntypes,
                  hipStream_t s);
void hx_embed_word_grad_sorted(int bf16, const void* dz, const int64_t* ids, const int64_t* order, float* dwte,
                               int64_t rows, int H, hipStream_t s);
// elementwise.hip
int hx_colsum_ws_floats(int64_t rows, int N);
void hx_bias_act_fwd(int bf16, int act, const void* y, const float* b, void* out, int64_t rows, int N, hipStream_t s);
void hx_bias_act_bwd(int bf16, int act, const void* dout, const void* y, const float* b, const void* saved_out,
                     void* dy, float* partial, float* dbias, int64_t rows, int N, int accumulate, hipStream_t s);
void hx_colsum(int bf16, void* x, const float* scale, float* partial, float* out, int64_t rows, int N, int accumulate,
               hipStream_t s, int64_t ld = -1);
void hx_dropout(int bf16, const void* x, void* out, int64_t n, float keep_prob, const uint64_t* seed, uint64_t stream,
                hipStream_t s);

// xent.hip
void hx_softmax_xent(int bf16, void* logits, const float* bias, const int64_t* labels, float* loss, int64_t rows,
                     int V, int64_t ld, int64_t ignore_index, hipStream_t s);

// attention.hip
size_t hx_attn_bwd_smem_bytes();
// bias: optional [3H] QKV-projection bias added to Q/K/V as they are loaded
void hx_attn_fwd_bf16(const void* qkv, const float* bias, const float* maskb, void* out, float* lse, uint32_t* dmask,
                      int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream, hipStream_t s);
void hx_attn_bwd_bf16(const void* qkv, const float* bias, float* dbias_part, const float* maskb, const void* dout,
                      const void* out, const float* lse, const uint32_t* dmask, void* dqkv, float* dq_acc, int dq_ld,
                      int B, int S, int nh, float keep, hipStream_t s);
// bf16 weight gradient dW[M][N] (fp32) = dY[T][M]^T . X[T][N] (wgrad_bf16.hip); ws: nsplit * M * N floats
void hx_wgrad_bf16_plan(int M, int N, int T, int* cfg, int* nsplit);
void hx_wgrad_bf16(const void* dy, int ldy, const void* x, int ldx, float* out, float* ws, int M, int N, int T,
                   int cfg, int nsplit, int mvalid, hipStream_t s);
// attention_f16.hip -- fp32 attention on the fp16 matrix cores (three passes over scaled two-piece
// operands: --fp32-gemm fp16x3); amax_part (optional): max |out| (forward) / max |dQKV| (backward,
// S <= 128) per (row, head), [B * S][nh] -- the fp16x3 GEMMs' per-row operand scales; colmax_part
// (optional): max |out| of each column per (batch, 128-query block), [B * ceil(S / 128)][H]
// (forward) / max |dQKV| of each column per batch, [B][3H] (backward, S <= 128) -- the weight
// gradients' per-column scales
void hx_attn_fwd_f16(const float* qkv, const float* bias, const float* maskb, float* out, float* lse,
                     uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream,
                     hipStream_t s, float* amax_part = nullptr, float* colmax_part = nullptr);
void hx_attn_bwd_f16(const float* qkv, const float* bias, float* dbias_part, const float* maskb, const float* dout,
                     const float* out, const float* lse, const uint32_t* dmask, float* dqkv, float* dq_acc, int dq_ld,
                     int B, int S, int nh, float keep, hipStream_t s, float* amax_part = nullptr,
                     float* colmax_part = nullptr);
void hx_attn_fwd(int bf16, const void* qkv, const float* bias, const float* maskb, void* out, float* lse,
                 uint32_t* dmask, int B, int S, int nh, float keep, const uint64_t* seed, uint64_t stream, hipStream_t s);
// dq_acc: fp32 dQ accumulation target when S > 128 (atomics; row stride dq_ld), else unused.
// With bias: its gradient (column sums of dQ / dK / dV) goes to dbq / dbk / dbv through the
// dbias_part workspace ([B * ceil(S/128)][3H] fp32).  kind: 0 fp32 MFMA, 1 bf16, 3 fp32 as fp16x3.
void hx_attn_bwd(int kind, const void* qkv, const float* bias, float* dbq, float* dbk, float* dbv, float* dbias_part,
                 const float* maskb, const void* dout, const void* out, const float* lse, const uint32_t* dmask,
                 void* dqkv, float* dq_acc, int dq_ld, int B, int S, int nh, float keep, hipStream_t s,
                 float* amax_part = nullptr, float* colmax_part = nullptr);

// a batch of weights prepared in one launch (gemm_f16.hip: split_weight_f16 / weight_bf16_t);
// start[i] = first 64 x 64 tile of weight i, start[n] = total tiles
#define HX_WBATCH 64
struct HxWeightBatch {
  int n;
  const float* W[HX_WBATCH];
  uint16_t* wf[HX_WBATCH];
  uint16_t* wt[HX_WBATCH];
  int N[HX_WBATCH], K[HX_WBATCH];
  int nv[HX_WBATCH];   // split_weight_f16: rows at or past nv read as zero (0: all N rows) -- padded vocabularies
  int start[HX_WBATCH + 1];
  int64_t roff[HX_WBATCH];   // split_weight_f16: weight i's row maxima [N] then column maxima [K] at rc + roff[i]
};
// fold [rows][N] column partials into out[N] (+= if accumulate)
void hx_fold_cols(const float* partial, int rows, int N, float* out, int accumulate, hipStream_t s);

// gemm_f16.hip -- --fp32-gemm fp16x3: fp32 operands as two scaled fp16 pieces, three MFMA passes.
// A: fp32 [M][K] (row stride lda, split in the kernel), B: fp16 pieces in the P2 layout [N][2K].
// Operand scales are per ROW of A and per row of B (= output column): row r's max |x| is the max
// of a_amax[r * a_rs + j], j < na (a_rs = 0: the same na partials for every row, a per-tensor
// bound); likewise b_amax / nb / b_rs.
// kind 0: C (+)= acc (+ bias)  [ks > 1: split-K slabs C + z c_zs, no bias / beta]
// kind 1: u = acc + bias -> C = gelu'(u) (dmode 1) or u (dmode 0); P = gelu(u) fp32
// kind 2: t = acc * (dmode ? aux : gelu'(aux + bias)) -> P fp32, colpart
//         [hx_gemm_f16_colpart_rows][N] per-wave column sums of t
// kinds 1 / 2 (optional): rowmax [M][hx_gemm_f16_tn] = max |P| per (row, N tile) -- the next
//         GEMM's row scale; colmax [hx_gemm_f16_tm][N] = max |P| per (M tile, column) -- the weight
//         gradient's column scale
struct HxGemmF16 {
  const void* A;     // fp32, or bf16 when abf16 (then B is bf16 [N][K] and there is no scaling)
  int64_t lda;
  const float* a_amax;
  int na, a_rs;
  const uint16_t* B;
  int64_t ldb;
  const float* b_amax;
  int nb, b_rs;
  float* C;
  int64_t ldc;
  int M, N, K, beta, kind;
  const float* bias;
  const float* aux;
  int64_t ldaux;
  float* P;
  int64_t ldp;
  float* colpart;
  float* rowmax;
  float* colmax;
  int dmode, ks;
  int64_t c_zs;
  int abf16, obf16;   // --precision bf16: bf16 operands (one pass), bf16 output C (kind 0)
  int apieces;        // A is fp16 P2 pieces [M][2K] split at its row scale (lda counts 4-B k slots)
};
// --precision bf16: W^T [K][N] bf16 of every weight of a batch (wt used, wf / mask ignored)
void hx_weight_bf16_t(const HxWeightBatch& d, hipStream_t s);
// fp32 rows [rows][K] (row stride ldx) -> fp16 P2 pieces [rows][2K] at each row's scale (max of np
// partials per row, amax[r np + j])
void hx_split_rows_f16(const float* x, int64_t ldx, const float* amax, int np, int64_t rows, int K, uint16_t* out,
                       hipStream_t s);
int hx_gemm_f16_plan(int M, int N, int K);
int hx_gemm_bf16_plan(int M, int N, int K);
int hx_gemm_f16_tiles(int M, int N, int cfg);
int hx_gemm_f16_tm(int M, int cfg);   // M tiles
int hx_gemm_f16_tn(int N, int cfg);   // N tiles
int hx_gemm_f16_colpart_rows(int M, int cfg);
int hx_gemm_f16_ks(int M, int N, int K, int cfg);
// split-K combine: C[M][ldc] (+= if beta) = sum of ks [M][N] slabs at ws (+ bias [N]); N % 4 == 0
void hx_gemm_f16_slab_combine(const float* ws, float* C, int64_t ldc, int M, int N, int ks, int beta,
                              const float* bias, hipStream_t s);
int hx_gemm_f16(const HxGemmF16& p, int cfg, hipStream_t s);
// dW[M][N] = dY[T][M]^T X[T][N] (fp32 operands, row strides ldy / ldx); rows >= mvalid not stored;
// ws: nsplit * M * N floats when nsplit > 1.  Operand scales per COLUMN (the non-reduction
// dimension), each operand's from an HxColScale: column c's max |x| is
//   g != null:  (|g[c]| z + |b[c]|) mul  (a bound: a LayerNorm output gamma zhat + beta, |zhat| <= z)
//   cs > 0:     max over j < np of p[j cs + c]  ([np][C] column partials)
//   cs == 0:    max over the np partials at p   (one per-tensor bound)
struct HxColScale {
  const float* p;
  int np, cs;
  const float* g;
  const float* b;
  float z, mul;
};
void hx_wgrad_f16_plan(int M, int N, int T, int* cfg, int* nsplit);
int hx_wgrad_f16(const float* dy, int ldy, const HxColScale& ca, const float* x, int ldx, const HxColScale& cb,
                 float* out, float* ws, int M, int N, int T, int cfg, int nsplit, int mvalid, hipStream_t s);
// max |x| of each column of a [rows][cols] fp32 matrix (cols % 4 == 0, 16-B rows) -> out[cols]
void hx_amax_cols(const float* x, int64_t rows, int cols, int64_t ld, float* out, hipStream_t s);
// max |x| of each row of a [rows][cols] fp32 matrix (cols % 4 == 0, 16-B rows) -> out[rows]
void hx_amax_rows(const float* x, int64_t rows, int cols, int64_t ld, float* out, hipStream_t s);
int hx_amax_rows_cols(const float* x, int64_t rows, int cols, int64_t ld, float* rowmax, float* colmax,
                      hipStream_t s);
// every weight of a batch -> P2 fp16 pieces wf [N][2K] (row n scaled by its own 2^E), wt [K][2N]
// (row k = column k of W, scaled by that column's 2^E); rc: per weight its row maxima [N] then
// column maxima [K] at rc + roff[i] (rc_floats in all, zeroed here)
void hx_split_weight_f16(const HxWeightBatch& d, float* rc, int64_t rc_floats, hipStream_t s);

// split.hip -- fp32 -> bf16 planes (piece order[j] = (order >> 4j) & 15) for bf16-MFMA
// emulation of fp32 GEMMs; interleaved [R][npl][D] or stacked [npl][R][D].
// Output rows padded to Rp (stacked) / columns to Dp with zeros.
void hx_split_planes(const float* x, int64_t ldx, uint16_t* out, int64_t R, int D, int64_t Rp, int Dp,
                     int npieces, int npl, uint32_t order, int stacked, hipStream_t s);
// Transposed weight planes [K][npl][Np]: out[k][j * Np + n] = piece order[j] of W[n][k]
// (n >= N zero-filled); K and Np multiples of 64, W rows 16-B aligned.
void hx_split_planes_t(const float* W, int64_t ldw, int N, int K, uint16_t* out, int Np, int npieces, int npl,
                       uint32_t order, hipStream_t s);

// xgmi_allreduce.hip -- intra-node in-place all-reduce (two-shot; one-shot for buckets up to
// oneshot_max_bytes) over IPC-mapped peer gradient buffers.  Sequence: create, register (the
// buffer every bucket is a slice of), export -> exchange -> open, then allreduce per bucket.
// Every function returns 0 on success, -1 with a message in hx_xar_last_error().
constexpr int kXarRecord = 192;   // exported bytes per rank
const char* hx_xar_last_error();
int hx_xar_create(int rank, int world, int nblocks, double timeout_s, int64_t oneshot_max_bytes, void** ctx);
int64_t hx_xar_oneshot_max(void* ctx);
int hx_xar_register(void* ctx, float* base, int64_t n);
int hx_xar_export(void* ctx, char* out);
int hx_xar_open(void* ctx, const char* recs);
int hx_xar_allreduce(void* ctx, float* buf, int64_t n, hipStream_t s);
// mute >= 0: that simulated rank never raises its flags (test hook: the others time out)
int hx_xar_allreduce_sim(void** ctxs, float** bufs, int W, int64_t n, int mute, hipStream_t s);
int hx_xar_error(void* ctx);
// stream-ordered copy of the error word into a device int32 (no host sync)
int hx_xar_error_async(void* ctx, int32_t* dst, hipStream_t s);
void hx_xar_destroy(void* ctx);

// cu_reserve.hip: CUs held back from the one-round GEMM plans for a concurrent comm kernel
int hx_num_cus();
void hx_set_reserved_cus(int r);
int hx_reserved_cus();
int hx_cu_slots();   // workgroup slots of one round: n_cu - reserved
hipStream_t hx_cu_masked_stream(int first_cu, int count);
hipStream_t hx_priority_stream(int prio);
void hx_stream_priority_range(int* least, int* greatest);
void hx_destroy_stream(hipStream_t s);
void hx_spin(int blocks, double us, int lds_bytes, uint32_t* sink, hipStream_t s);
