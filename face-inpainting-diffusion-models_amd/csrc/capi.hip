// extern "C" entry points of libifd.so (declared in include/ifd.h).
#include <cstring>
#include <new>
#include <string>

#include "unet.h"

static_assert(sizeof(ifd_step_coeffs) == sizeof(ifd::StepCoeffs), "coefficient struct layout");

namespace ifd {
static thread_local std::string g_err;
void set_error(const std::string& m) { g_err = m; }
const char* get_error() { return g_err.c_str(); }
void clear_error() { g_err.clear(); }
}  // namespace ifd

struct ifd_handle {
  ifd::Model* model;
};

using ifd::set_error;

extern "C" {

const char* ifd_last_error(void) { return ifd::get_error(); }
void ifd_clear_error(void) { ifd::clear_error(); }
const char* ifd_version(void) { return "ifd 0.2 gfx950 fp32-mfma + 3xf16-split-mfma"; }

int ifd_create(const ifd_config* cfg, ifd_handle** out) {
  if (!cfg || !out) {
    set_error("ifd_create: null argument");
    return 2;
  }
  if (cfg->num_levels < 1 || cfg->num_levels > 8 || cfg->model_channels % 32 != 0 || cfg->in_channels > 16 ||
      cfg->num_res_blocks < 1 || (cfg->image_size >> (cfg->num_levels - 1)) < 2 || cfg->out_channels > 32 ||
      cfg->out_channels % 2 != 0) {
    set_error("ifd_create: unsupported configuration");
    return 2;
  }
  try {
    *out = new ifd_handle{new ifd::Model(*cfg)};
  } catch (const std::exception& e) {
    set_error(std::string("ifd_create: ") + e.what());
    return 1;
  }
  return 0;
}

void ifd_destroy(ifd_handle* h) {
  if (!h) return;
  delete h->model;
  delete h;
}

int ifd_num_params(ifd_handle* h, int* n) {
  if (!h || !n) { set_error("null argument"); return 2; }
  *n = (int)h->model->params().size();
  return 0;
}

int ifd_param_info(ifd_handle* h, int i, const char** name, int64_t* shape4, int* ndim) {
  if (!h) { set_error("null handle"); return 2; }
  const auto& ps = h->model->params();
  if (i < 0 || i >= (int)ps.size()) { set_error("param index out of range"); return 2; }
  if (name) *name = ps[i].name.c_str();
  if (ndim) *ndim = (int)ps[i].shape.size();
  if (shape4)
    for (int k = 0; k < 4; ++k) shape4[k] = k < (int)ps[i].shape.size() ? ps[i].shape[k] : 1;
  return 0;
}

int ifd_load_weights(ifd_handle* h, const char* name, const float* data, const int64_t* shape, int ndim) {
  if (!h || !name || !data || !shape) { set_error("ifd_load_weights: null argument"); return 2; }
  return h->model->load(name, data, shape, ndim);
}

int ifd_finalize(ifd_handle* h) {
  if (!h) { set_error("null handle"); return 2; }
  return h->model->finalize();
}

int ifd_set_precision(ifd_handle* h, int prec) {
  if (!h) { set_error("null handle"); return 2; }
  return h->model->set_precision(prec);
}

int ifd_get_precision(ifd_handle* h, int* prec) {
  if (!h || !prec) { set_error("null argument"); return 2; }
  *prec = h->model->precision();
  return 0;
}

int ifd_guard_reset(ifd_handle* h, void* stream) {
  if (!h) { set_error("null handle"); return 2; }
  return h->model->guard_reset((hipStream_t)stream);
}

int ifd_guard_read(ifd_handle* h, int* tripped, void* stream) {
  if (!h || !tripped) { set_error("ifd_guard_read: null argument"); return 2; }
  return h->model->guard_read((hipStream_t)stream, tripped);
}

int ifd_guard_copy_async(ifd_handle* h, unsigned* host_dst, void* stream) {
  if (!h || !host_dst) { set_error("ifd_guard_copy_async: null argument"); return 2; }
  return h->model->guard_copy_async((hipStream_t)stream, host_dst);
}

int ifd_set_option(ifd_handle* h, const char* key, int value) {
  if (!h || !key) { set_error("ifd_set_option: null argument"); return 2; }
  return h->model->set_option(key, value);
}

int ifd_get_option(ifd_handle* h, const char* key, int* value) {
  if (!h || !key || !value) { set_error("ifd_get_option: null argument"); return 2; }
  return h->model->get_option(key, value);
}

int ifd_memory(ifd_handle* h, int64_t* wb, int64_t* ws) {
  if (!h) { set_error("null handle"); return 2; }
  if (wb) *wb = h->model->weight_bytes();
  if (ws) *ws = h->model->workspace_bytes();
  return 0;
}

int ifd_workspace_plan(ifd_handle* h, int64_t B, int64_t* ws) {
  if (!h || !ws || B < 1 || B > (1 << 20)) { set_error("ifd_workspace_plan: bad argument"); return 2; }
  *ws = h->model->workspace_bytes_for((int)B);
  return 0;
}

int ifd_profile_enable(ifd_handle* h, int on) {
  if (!h) { set_error("null handle"); return 2; }
  return h->model->profile_enable(on);
}

int ifd_profile_filter(ifd_handle* h, const char* prefix) {
  if (!h) { set_error("null handle"); return 2; }
  return h->model->profile_filter(prefix);
}

int ifd_profile_report(ifd_handle* h, char* buf, int64_t buflen) {
  if (!h || !buf || buflen <= 0) { set_error("ifd_profile_report: bad argument"); return 2; }
  std::string js;
  if (h->model->profile_report(js)) return 1;
  if ((int64_t)js.size() + 1 > buflen) { set_error("ifd_profile_report: buffer too small"); return 2; }
  std::memcpy(buf, js.c_str(), js.size() + 1);
  return 0;
}

int ifd_unet_forward(ifd_handle* h, const float* x, const float* masked_image, const float* mask, const int64_t* t,
                     int64_t B, int H, int W, float* out6, void* stream) {
  if (!h || !x || !masked_image || !mask || !t || !out6) { set_error("ifd_unet_forward: null argument"); return 2; }
  return h->model->forward(x, masked_image, mask, 0, t, (int)B, H, W, ifd::EPI_NCHW, out6, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr, (hipStream_t)stream);
}

static int step_common(ifd_handle* h, int epi, const int64_t* t, int64_t B, int H, int W, float* img, const float* gt,
                       const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c,
                       void* stream) {
  if (!h || !t || !img || !gt || !mask || !c) { set_error("ifd step: null argument"); return 2; }
  if (c->inject && !known) { set_error("ifd step: inject requires known noise"); return 2; }
  if (epi == ifd::EPI_DDIM && c->use_noise && !noise) { set_error("ifd_ddim_step: use_noise requires noise"); return 2; }
  if (epi == ifd::EPI_DDPM && !noise) { set_error("ifd_ddpm_step: noise required"); return 2; }
  ifd::StepCoeffs sc;
  std::memcpy(&sc, c, sizeof(sc));
  return h->model->forward(img, gt, mask, 1, t, (int)B, H, W, epi, nullptr, &sc, img, gt, mask, noise, known,
                           (hipStream_t)stream);
}

int ifd_ddim_step(ifd_handle* h, const int64_t* t, int64_t B, int H, int W, float* img, const float* gt,
                  const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c, void* stream) {
  return step_common(h, ifd::EPI_DDIM, t, B, H, W, img, gt, mask, noise, known, c, stream);
}

int ifd_ddpm_step(ifd_handle* h, const int64_t* t, int64_t B, int H, int W, float* img, const float* gt,
                  const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c, void* stream) {
  return step_common(h, ifd::EPI_DDPM, t, B, H, W, img, gt, mask, noise, known, c, stream);
}

static int update_common(int mode, const float* out6, int64_t B, int H, int W, float* img, const float* gt,
                         const float* mask, const float* noise, const float* known, const ifd_step_coeffs* c,
                         void* stream) {
  if (B < 0 || H <= 0 || W <= 0 || !c) { set_error("ifd update: bad shape or null coefficients"); return 2; }
  if (B == 0) return 0;  /* an empty batch: nothing to launch (a zero-size grid is a launch error) */
  if (!out6 || !img) { set_error("ifd update: null argument"); return 2; }
  if (c->inject && (!gt || !mask || !known)) { set_error("ifd update: inject requires gt, mask, known"); return 2; }
  if ((mode == ifd::EPI_DDPM || c->use_noise) && !noise) { set_error("ifd update: noise required"); return 2; }
  ifd::StepCoeffs sc;
  std::memcpy(&sc, c, sizeof(sc));
  ifd::launch_step(mode, sc, out6, img, gt, mask, noise, known, (int)B, H * W, (hipStream_t)stream);
  return ifd::launch_status(mode == ifd::EPI_DDPM ? "ifd_ddpm_update" : "ifd_ddim_update") ? 1 : 0;
}

int ifd_ddim_update(const float* out6, int64_t B, int H, int W, float* img, const float* gt, const float* mask,
                    const float* noise, const float* known, const ifd_step_coeffs* c, void* stream) {
  return update_common(ifd::EPI_DDIM, out6, B, H, W, img, gt, mask, noise, known, c, stream);
}

int ifd_ddpm_update(const float* out6, int64_t B, int H, int W, float* img, const float* gt, const float* mask,
                    const float* noise, const float* known, const ifd_step_coeffs* c, void* stream) {
  return update_common(ifd::EPI_DDPM, out6, B, H, W, img, gt, mask, noise, known, c, stream);
}

int ifd_blend(const float* result, const float* gt, const float* mask, int64_t B, int C, int H, int W, float* out,
              void* stream) {
  if (B < 0 || C <= 0 || H <= 0 || W <= 0) { set_error("ifd_blend: bad shape"); return 2; }
  if (B == 0) return 0;  /* an empty batch: nothing to launch */
  if (!result || !gt || !mask || !out) { set_error("ifd_blend: null argument"); return 2; }
  ifd::launch_blend(result, gt, mask, out, (int)B, C, H * W, (hipStream_t)stream);
  return IFD_LAUNCH_STATUS() ? 1 : 0;
}

int ifd_to_u8(const float* sample, int64_t B, int C, int H, int W, uint8_t* out_nhwc, void* stream) {
  if (B < 0 || C <= 0 || H <= 0 || W <= 0 || B * H * W > INT32_MAX) { set_error("ifd_to_u8: bad shape"); return 2; }
  if (B == 0) return 0;  /* an empty tensor may carry a null pointer */
  if (!sample || !out_nhwc) { set_error("ifd_to_u8: null argument"); return 2; }
  ifd::launch_to_u8(sample, out_nhwc, (int)B, C, H * W, (hipStream_t)stream);
  return IFD_LAUNCH_STATUS() ? 1 : 0;
}

int ifd_mask_from_gray(const uint8_t* gray, int64_t n, float* mask, void* stream) {
  if (n < 0 || ((!gray || !mask) && n > 0)) { set_error("ifd_mask_from_gray: bad argument"); return 2; }
  if (n == 0) return 0;
  ifd::launch_mask_from_gray(gray, mask, n, (hipStream_t)stream);
  return IFD_LAUNCH_STATUS() ? 1 : 0;
}

}  // extern "C"
