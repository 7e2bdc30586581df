// Input-side data formats of the sampler and the trainer: the dataset's
// transforms moved onto the GPU so a batch is assembled without host work per image.
//   * ifd_resize_u8: Pillow's BILINEAR resample of 8-bit images (what torchvision's
//     transforms.Resize((s, s)) does to the dataset's PIL images, code/data/dataset.py:231-240),
//     bit-exact: Resample.c's coefficients (triangle filter, support max(1, scale), normalised,
//     22-bit fixed point), a horizontal pass over the rows the vertical pass needs, then the
//     vertical pass, each rounding to uint8 with Pillow's clip.
//   * ifd_image_to_float: ToTensor + Normalize([0.5]*3, [0.5]*3) (dataset.py:238-240), NHWC u8 ->
//     NCHW fp32 in [-1, 1].
//   * ifd_make_inpaint_batch: OrderedMaskDataset.__getitem__'s mask part (dataset.py:273-286) for
//     a whole batch: mask = bank[idx % M] thresholded (< 0.5 after /255: 1 = hole),
//     masked_image = image * (1 - mask).
// All byte / elementwise work: HBM-bound, one thread per output value, coalesced along the
// innermost (channel, then x) dimension.
#include <cmath>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

#include "../../include/ifd.h"
#include "common.h"

namespace ifd {
namespace {

constexpr int PB = 32 - 8 - 2;  // Pillow's PRECISION_BITS

// Resample.c precompute_coeffs (bilinear filter) + normalize_coeffs_8bpc, in double as Pillow does.
int resize_coeffs_host(int in_size, int out_size, std::vector<int>& bounds, std::vector<int>& kk) {
  const double scale = (double)in_size / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  bounds.assign((size_t)out_size * 2, 0);
  kk.assign((size_t)out_size * ksize, 0);
  std::vector<double> w(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = (xx + 0.5) * scale;
    const double ss = 1.0 / filterscale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      w[x] = t < 1.0 ? 1.0 - t : 0.0;
      ww += w[x];
    }
    for (int x = 0; x < xmax; ++x) {
      const double v = ww != 0.0 ? w[x] / ww : w[x];
      kk[(size_t)xx * ksize + x] = v < 0 ? (int)(-0.5 + v * (1 << PB)) : (int)(0.5 + v * (1 << PB));
    }
    bounds[(size_t)xx * 2] = xmin;
    bounds[(size_t)xx * 2 + 1] = xmax;
  }
  return ksize;
}

struct DevCoeffs {
  int* bounds = nullptr;
  int* kk = nullptr;
  int ksize = 0;
  int first = 0, last = 0;  // rows/cols of the input the pass reads
};

// device copies of the coefficient tables, cached per (device, in, out)
std::mutex g_coeff_mu;
std::map<std::tuple<int, int, int>, DevCoeffs> g_coeffs;

int get_coeffs(int in_size, int out_size, DevCoeffs* out) {
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_coeff_mu);
  auto key = std::make_tuple(dev, in_size, out_size);
  auto it = g_coeffs.find(key);
  if (it != g_coeffs.end()) {
    *out = it->second;
    return 0;
  }
  std::vector<int> b, k;
  DevCoeffs d;
  d.ksize = resize_coeffs_host(in_size, out_size, b, k);
  d.first = b[0];
  d.last = b[(size_t)(out_size - 1) * 2] + b[(size_t)(out_size - 1) * 2 + 1];
  IFD_CHECK_HIP(hipMalloc(&d.bounds, b.size() * sizeof(int)));
  IFD_CHECK_HIP(hipMalloc(&d.kk, k.size() * sizeof(int)));
  IFD_CHECK_HIP(hipMemcpy(d.bounds, b.data(), b.size() * sizeof(int), hipMemcpyHostToDevice));
  IFD_CHECK_HIP(hipMemcpy(d.kk, k.data(), k.size() * sizeof(int), hipMemcpyHostToDevice));
  g_coeffs[key] = d;
  *out = d;
  return 0;
}

__device__ __forceinline__ unsigned char clip8(int in) {
  if (in >= (1 << PB << 8)) return 255;
  if (in <= 0) return 0;
  return (unsigned char)(in >> PB);
}

// horizontal pass: out[n][y][xx][c] = sum_x in[n][y0 + y][xmin + x][c] * k[xx][x], y in [0, rows)
__global__ void resample_h_kernel(const unsigned char* __restrict__ in, int Hin, int Win, int C, int y0, int rows,
                                  int Wout, const int* __restrict__ bounds, const int* __restrict__ kk, int ksize,
                                  unsigned char* __restrict__ out, int64_t tot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int c = (int)(i % C);
  int64_t r = i / C;
  const int xx = (int)(r % Wout);
  r /= Wout;
  const int y = (int)(r % rows);
  const int64_t n = r / rows;
  const int xmin = bounds[2 * xx], xmax = bounds[2 * xx + 1];
  const unsigned char* row = in + ((n * Hin + y0 + y) * (int64_t)Win) * C + c;
  int ss = 1 << (PB - 1);
  for (int x = 0; x < xmax; ++x) ss += (int)row[(int64_t)(xmin + x) * C] * kk[xx * ksize + x];
  out[i] = clip8(ss);
}

// vertical pass over an image of `Hsrc` rows: out[n][yy][x][c] = sum_y in[n][ymin + y][x][c] * k[yy][y]
__global__ void resample_v_kernel(const unsigned char* __restrict__ in, int Hsrc, int W, int C, int Hout,
                                  const int* __restrict__ bounds, const int* __restrict__ kk, int ksize, int yshift,
                                  unsigned char* __restrict__ out, int64_t tot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= tot) return;
  const int64_t WC = (int64_t)W * C;
  const int64_t xc = i % WC;
  int64_t r = i / WC;
  const int yy = (int)(r % Hout);
  const int64_t n = r / Hout;
  const int ymin = bounds[2 * yy] - yshift, ymax = bounds[2 * yy + 1];
  const unsigned char* col = in + (n * Hsrc) * WC + xc;
  int ss = 1 << (PB - 1);
  for (int y = 0; y < ymax; ++y) ss += (int)col[(int64_t)(ymin + y) * WC] * kk[yy * ksize + y];
  out[i] = clip8(ss);
}

__global__ void copy_u8_kernel(const unsigned char* __restrict__ a, unsigned char* __restrict__ b, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = a[i];
}

// ToTensor (x / 255, fp32) + Normalize(0.5, 0.5): (v - 0.5) / 0.5; NHWC u8 -> NCHW fp32
__global__ void image_to_float_kernel(const unsigned char* __restrict__ src, int C, int HW, float* __restrict__ dst,
                                      int64_t tot) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // NCHW output index
  if (i >= tot) return;
  const int64_t p = i % HW;
  const int64_t nc = i / HW;
  const int c = (int)(nc % C);
  const int64_t n = nc / C;
  const float v = (float)src[(n * HW + p) * C + c] / 255.0f;
  dst[i] = (v - 0.5f) / 0.5f;
}

// mask[n][p] = (bank[idx[n] % M][p] / 255 < 0.5); masked[n][c][p] = image[n][c][p] * (1 - mask)
__global__ void inpaint_batch_kernel(const float* __restrict__ images, int HW, const unsigned char* __restrict__ bank,
                                     int M, const int64_t* __restrict__ idx, float* __restrict__ mask,
                                     float* __restrict__ masked, int64_t npix) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (n, p)
  if (i >= npix) return;
  const int64_t n = i / HW, p = i % HW;
  int64_t k = idx[n] % M;
  if (k < 0) k += M;
  const float g = (float)bank[k * HW + p] / 255.0f;
  const float m = g < 0.5f ? 1.0f : 0.0f;
  if (mask) mask[i] = m;
  if (masked) {
    const float keep = 1.0f - m;
    for (int c = 0; c < 3; ++c) {
      const int64_t o = (n * 3 + c) * HW + p;
      masked[o] = images[o] * keep;
    }
  }
}

}  // namespace
}  // namespace ifd

using namespace ifd;

extern "C" {

int ifd_resize_coeffs(int in_size, int out_size, int* bounds, int* coeffs, int* ksize) {
  if (in_size <= 0 || out_size <= 0 || !ksize) { set_error("ifd_resize_coeffs: bad arguments"); return 2; }
  std::vector<int> b, k;
  *ksize = resize_coeffs_host(in_size, out_size, b, k);
  if (bounds) std::copy(b.begin(), b.end(), bounds);
  if (coeffs) std::copy(k.begin(), k.end(), coeffs);
  return 0;
}

int64_t ifd_resize_u8_workspace(int64_t N, int C, int Hin, int Win, int Hout, int Wout) {
  if (N <= 0 || C <= 0 || Hin <= 0 || Win <= 0 || Hout <= 0 || Wout <= 0) return 0;
  if (Wout == Win) return 0;
  std::vector<int> b, k;
  resize_coeffs_host(Hin, Hout, b, k);
  const int rows = b[(size_t)(Hout - 1) * 2] + b[(size_t)(Hout - 1) * 2 + 1] - b[0];
  return N * rows * (int64_t)Wout * C;
}

int ifd_resize_u8(const uint8_t* src, int64_t N, int C, int Hin, int Win, int Hout, int Wout, uint8_t* dst,
                  uint8_t* work, int64_t work_bytes, void* stream) {
  if (N < 0 || C <= 0 || Hin <= 0 || Win <= 0 || Hout <= 0 || Wout <= 0) {
    set_error("ifd_resize_u8: bad shape");
    return 2;
  }
  if (N == 0) return 0;
  if (!src || !dst) { set_error("ifd_resize_u8: null argument"); return 2; }
  hipStream_t s = (hipStream_t)stream;
  const bool need_h = Wout != Win, need_v = Hout != Hin;
  if (!need_h && !need_v) {
    const int64_t n = N * Hin * (int64_t)Win * C;
    hipLaunchKernelGGL(copy_u8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
    return IFD_LAUNCH_STATUS();
  }
  DevCoeffs cv, ch;
  if (get_coeffs(Hin, Hout, &cv)) return 1;
  const uint8_t* vin = src;
  int vrows = Hin, yshift = 0;
  if (need_h) {
    if (get_coeffs(Win, Wout, &ch)) return 1;
    const int rows = need_v ? cv.last - cv.first : Hin;
    const int64_t tot = N * rows * (int64_t)Wout * C;
    uint8_t* tmp = need_v ? work : dst;
    if (need_v && (!work || tot > work_bytes)) {
      set_error("ifd_resize_u8: workspace too small (ifd_resize_u8_workspace)");
      return 2;
    }
    hipLaunchKernelGGL(resample_h_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, src, Hin, Win, C,
                       need_v ? cv.first : 0, need_v ? rows : Hin, Wout, ch.bounds, ch.kk, ch.ksize, tmp, tot);
    vin = tmp;
    vrows = rows;
    yshift = cv.first;
  }
  if (need_v) {
    const int64_t tot = N * Hout * (int64_t)Wout * C;
    hipLaunchKernelGGL(resample_v_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, vin, vrows, Wout, C,
                       Hout, cv.bounds, cv.kk, cv.ksize, yshift, dst, tot);
  }
  return IFD_LAUNCH_STATUS();
}

int ifd_image_to_float(const uint8_t* src_nhwc, int64_t N, int C, int H, int W, float* dst_nchw, void* stream) {
  if (N < 0 || C <= 0 || H <= 0 || W <= 0) { set_error("ifd_image_to_float: bad shape"); return 2; }
  const int64_t tot = N * C * (int64_t)H * W;
  if (tot == 0) return 0;
  if (!src_nhwc || !dst_nchw) { set_error("ifd_image_to_float: null argument"); return 2; }
  hipLaunchKernelGGL(image_to_float_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     src_nhwc, C, H * W, dst_nchw, tot);
  return IFD_LAUNCH_STATUS();
}

int ifd_make_inpaint_batch(const float* images, int64_t N, int H, int W, const uint8_t* mask_bank, int M,
                           const int64_t* idx, float* mask, float* masked_image, void* stream) {
  if (N < 0 || H <= 0 || W <= 0 || M <= 0) { set_error("ifd_make_inpaint_batch: bad shape"); return 2; }
  const int64_t npix = N * (int64_t)H * W;
  if (npix == 0) return 0;
  if (!mask_bank || !idx || (masked_image && !images)) { set_error("ifd_make_inpaint_batch: null argument"); return 2; }
  hipLaunchKernelGGL(inpaint_batch_kernel, dim3((unsigned)((npix + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     images, H * W, mask_bank, M, idx, mask, masked_image, npix);
  return IFD_LAUNCH_STATUS();
}

}  // extern "C"
