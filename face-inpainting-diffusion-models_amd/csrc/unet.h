// 9-channel ADM UNet execution plan (code/unet.py:14-200) on the HIP kernels.
#pragma once
#include <map>
#include <string>
#include <vector>

#include "../../include/ifd.h"
#include "kernels.h"

namespace ifd {

struct ConvW {
  int cin = 0, cin_pad = 0, cout = 0, cout_pad = 0, bn = 0, taps = 9;
  size_t w_off = 0, b_off = 0;     // float offsets in the device weight blob
  int cs = 0, cs_pad = 0;          // 1x1 skip segment input channels
  size_t ws_off = 0;
  bool has_skip = false;
  size_t x3_off = 0;   // float offset of the 3xf16 split packing (pack_conv_x3), 0 if none
  size_t x3s_off = 0;  // ... of the 1x1 skip segment
  bool x3_ok = false;  // every weight within the split's range (|w| < 32): the layer may run 3xf16
  size_t head_off = 0;  // float offset of the output-head packing (conv_head.hip), 0 if none
  size_t head_x3_off = 0;  // the 3xf16 head's split packing (conv_head_x3_pack), 0 if none
  bool head_x3_ok = false;  // every head weight within the split's range
  // the skip segment as its own launch (skip_x3.hip) in the split modes: split 1x1 packing, the
  // conv's own bias and the skip bias apart (b_off holds their sum for the fused kernels)
  size_t sk_off = 0, bmain_off = 0, sbias_off = 0;
  int sk_ntc = 0;
  bool sk_ok = false;
  std::string wname, bname, swname, sbname;  // source parameter names
};

struct GNW {
  size_t g_off = 0, b_off = 0;
  int C = 0;
  std::string prefix;
};

struct ResP {
  std::string prefix;
  int cin = 0, cout = 0, c_cat = 0;  // c_cat: channels of the concatenated skip tensor (output blocks)
  int xf = XF_NONE;
  GNW gn1, gn2;
  ConvW conv1, conv2;
  ConvW conv2_res;  // conv2 without its skip segment (bias = conv2's own): the separate-skip plan
  int emb_off = 0;
};

struct AttnP {
  std::string prefix;
  int C = 0;
  GNW gn;
  ConvW qkv, proj;
};

enum LayerKind { L_RES = 0, L_ATTN = 1 };
struct LayerP {
  int kind;
  int idx;
  int res_in;  // spatial size at input
};

struct ParamSpec {
  std::string name;
  std::vector<int64_t> shape;
};

class Model {
 public:
  explicit Model(const ifd_config& cfg);
  ~Model();

  const std::vector<ParamSpec>& params() const { return params_; }
  int load(const std::string& name, const float* data, const int64_t* shape, int ndim);
  int finalize();
  int forward(const float* x, const float* a, const float* m, int pack_mode, const int64_t* t, int B, int H, int W,
              int epi, float* out6, const StepCoeffs* sc, float* img, const float* gt, const float* mask,
              const float* noise, const float* known, hipStream_t s);
  int64_t weight_bytes() const { return (int64_t)wblob_floats_ * 4; }
  // Event-based per-launch profiler (records on the launch stream; read after a sync).
  int profile_enable(int on);
  int profile_filter(const char* prefix);  // record only launches whose name starts with prefix ("" = all)
  int profile_report(std::string& json);
  int64_t workspace_bytes() const { return (int64_t)ws_floats_ * 4; }
  // arena size a forward at batch B would allocate (host-side plan, no device memory touched)
  int64_t workspace_bytes_for(int B) const;
  // Conv arithmetic: IFD_PREC_FP32 (exact fp32 MFMA) or IFD_PREC_3XF16 (split f16 MFMA, fp32-accurate)
  int set_precision(int prec);
  int precision() const { return prec_; }
  // Handle options (ifd_set_option): initial values come from the environment once, at creation
  // (IFD_CONV_STREAM, IFD_X3_OFF, IFD_GN_FUSED, IFD_SKIP_SEP, IFD_BATCH_INVARIANT); nothing is read from
  // the environment per launch.
  int set_option(const std::string& key, int value);
  int get_option(const std::string& key, int* value) const;

 private:
  void build_plan();
  void add_param(const std::string& n, std::vector<int64_t> shape);
  int ensure_workspace(int B);
  int run_res(const ResP& r, const float* in0, int c0, const float* in1, int c1, int N, int Hin, float* out,
              hipStream_t s);
  int run_attn(const AttnP& a, const float* in, int N, int Hin, float* out, hipStream_t s);
  // GroupNorm coefficients A/B of cat(in0, in1) from the sources' granule statistics (fused into
  // the producing conv's epilogue when it could, else one gn_granules pass per source)
  int run_gn(const float* in0, int c0, const float* in1, int c1, int N, int HW, const GNW& gn, const float* emb,
             int emb_stride, int emb_off, float* A, float* B, hipStream_t s);
  struct StatRec {
    float* part = nullptr;
    int E = 0;
    float cnt = 0.f;
    int C = 0;
  };
  int stats_for(const float* buf, int C, int N, int HW, StatRec* out, hipStream_t s);
  int run_conv(const ConvW& cw, const float* in0, int c0, const float* in1, int c1, int N, int Hin, int H, int xf,
               int act, const float* A, const float* Bc, const float* s0, int sc0, const float* s1, int sc1,
               const float* res, int res_xf, int resH, float* out, int epi, hipStream_t s,
               const StepCoeffs* sc = nullptr, float* img = nullptr, const float* gt = nullptr,
               const float* mask = nullptr, const float* noise = nullptr, const float* known = nullptr);

  struct ProfRec {
    std::string name;
    double flops, bytes;
    hipEvent_t e0, e1;
  };
  bool prof_on_ = false;
  bool prof_layers_ = false;  // profile_enable(h, 2): key conv launches by layer shape
  std::string prof_filter_;
  std::vector<ProfRec> prof_;
  std::vector<hipEvent_t> ev_pool_;
  size_t ev_used_ = 0;
  hipEvent_t take_event();
  void prof_begin(hipStream_t s, hipEvent_t* e0, const char* name);
  void prof_end(hipStream_t s, hipEvent_t e0, const std::string& name, double flops, double bytes);

  ifd_config cfg_;
  std::vector<ParamSpec> params_;
  std::map<std::string, std::vector<float>> host_;  // loaded parameters (host copies until finalize)

  // plan
  ConvW conv_in_, conv_out_;
  GNW gn_out_;
  std::vector<ResP> res_;
  std::vector<AttnP> attn_;
  std::vector<std::vector<LayerP>> in_blocks_, out_blocks_;
  std::vector<LayerP> mid_;
  std::vector<int> in_ch_, in_res_;  // channels / resolution of each input block's output
  int emb_dim_ = 0, emb_total_ = 0;
  size_t te_w0_ = 0, te_b0_ = 0, te_w2_ = 0, te_b2_ = 0, freqs_ = 0, embw_ = 0, embb_ = 0;

  // device memory
  float* wblob_ = nullptr;
  size_t wblob_floats_ = 0;
  bool finalized_ = false;
  float* ws_ = nullptr;
  size_t ws_floats_ = 0;
  int ws_B_ = 0;
  // workspace carve (float offsets), valid for ws_B_
  struct WsLayout {
    size_t o_x0_ = 0, o_bufs_[3] = {0, 0, 0}, o_t1_ = 0, o_qkv_ = 0, o_ao_ = 0, o_A_ = 0, o_B_ = 0, o_part_ = 0,
           o_emb_ = 0, o_h1_ = 0, o_E_ = 0, o_split_ = 0, o_pool_ = 0, o_pool2_ = 0;
    size_t split_floats_ = 0;  // split-K slab capacity
    size_t pool_floats_ = 0;   // act_pool / act_apply staging capacity
    std::vector<size_t> o_hs_;
  };
  WsLayout ly_;
  size_t plan_workspace(int B, WsLayout& w, std::vector<std::pair<size_t, size_t>>& stat_of) const;
  // GroupNorm granule statistics: one area per activation buffer (hs, bufs, t1); stat_ holds the
  // buffers whose current contents have valid statistics (reset per forward)
  std::map<const float*, float*> stat_area_;
  std::map<const float*, StatRec> stat_;
  bool gn_fused_ = true;
  int opt_stream_ = 2;      // wide fp32 layers: 0 one tile per workgroup, 1/2 persistent (1 or 2 per CU)
  int opt_x3_off_ = 0;      // bisecting mask: 1 no 16x16 tiles, 2 no split-K, 4 no skip layers, 8 no 8x8, 16 no 1x1,
                            // 32 no split-MFMA output head
  int opt_invariant_ = 0;   // batch-invariant geometry (results independent of the batch split)
  int opt_skip_sep_ = 64;   // split modes: ResBlock skip_connection as its own launch at resolutions >= this (0 off)
  void fill_opts(ConvParams& p) const {
    p.opt_bm128 = 0;
    p.opt_invariant = opt_invariant_;
    p.opt_img8_partial = 1;
  }
  const float* pooled_raw_ = nullptr;  // tensor whose raw 2x2 pool sits in o_pool2_ (act_pool)
  int prec_ = 0;
  unsigned* guard_ = nullptr;  // 3xf16 range guard word (ConvParams::guard)

 public:
  // range guard: async reset / synchronous read (0 = every split operand was in range)
  int guard_reset(hipStream_t s);
  int guard_read(hipStream_t s, int* tripped);
  int guard_copy_async(hipStream_t s, unsigned* host_dst);
};

}  // namespace ifd
