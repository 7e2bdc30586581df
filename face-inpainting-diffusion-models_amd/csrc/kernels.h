// Host-side launchers of the non-conv kernels.
#pragma once
#include "conv.h"

namespace ifd {

int gn_slices(int HW, int* slice);
int launch_gn(const float* p0, int c0, const float* p1, int c1, int N, int HW, const float* gamma, const float* beta,
              const float* emb, int emb_stride, int emb_off, float* part, float* A, float* B, hipStream_t stream);
// granule statistics (norm.hip): P[N][C/4][E][2] = (mean, M2) over `cnt` values per entry
int launch_gn_granules(const float* x, int C, int N, int HW, float* part, int* E, float* cnt, hipStream_t stream);
int launch_gn_finalize2(const float* part0, int E0, float cnt0, int C0, const float* part1, int E1, float cnt1,
                        int C1, int N, const float* gamma, const float* beta, const float* emb, int emb_stride,
                        int emb_off, float* A, float* B, hipStream_t stream);
void launch_pack_input(const float* x, const float* a, const float* m, int mode, int N, int HW, float* out,
                       hipStream_t s);
void launch_temb(const int64_t* t, const float* freqs, int mc, const float* w0t, const float* b0, const float* w2t,
                 const float* b2, int E, int N, float* h1, float* emb, hipStream_t s);
void launch_emb_proj(const float* emb, int E, int N, const float* wt, const float* b, int J, float* out,
                     hipStream_t s);
void launch_attention(const float* qkv, int N, int T, int C, float scale, float* out, hipStream_t s);
void launch_step(int mode, const StepCoeffs& sc, const float* out6, float* img, const float* gt, const float* mask,
                 const float* noise, const float* known, int N, int HW, hipStream_t s);
// act + AvgPool2d(2,2) of an NHWC tensor (the down-ResBlock's h_upd, code/nn.py:190-195) for the
// split-precision conv, which has no avg-pool prologue: out[n, y, x, c] = ((a00 + a01) + a10) + a11) / 4
// with a = act(A[n,c] v + B[n,c]), the arithmetic of conv.hip's XF_DOWN prologue.
// act(A x + B) of an NHWC tensor (no pooling): the split kernel's 1x1 operand
int launch_act_apply(const float* x, int C, int N, int HW, int act, const float* A, const float* B, float* out,
                     hipStream_t s);
// out_raw (optional): also pool(x) without the act, from the same reads (the block's residual)
int launch_act_pool(const float* x, int C, int N, int Hin, int act, const float* A, const float* B, float* out,
                    float* out_raw, hipStream_t s);
void launch_blend(const float* res, const float* gt, const float* mask, float* out, int N, int C, int HW,
                  hipStream_t s);
void launch_to_u8(const float* x, unsigned char* out, int N, int C, int HW, hipStream_t s);
void launch_mask_from_gray(const unsigned char* g, float* m, int64_t n, hipStream_t s);

}  // namespace ifd
