// UNet plan, weight packing and forward orchestration (host side of the HIP library).
//
// Plan mirrors UNetModel.__init__ (code/unet.py:43-152) with resblock_updown=True,
// use_scale_shift_norm=True and the 9-channel first conv of DiffusionInpaintingModel
// (code/unet.py:184-188). Activations are NHWC fp32 in one workspace arena; skip tensors of the
// input blocks stay resident until the matching output block consumes them (no torch.cat: the
// conv reads the two sources by channel range).
#include "unet.h"

#include <algorithm>
#include <array>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace ifd {

static int ceil_to(int v, int m) { return (v + m - 1) / m * m; }

static int env_int(const char* name, int dflt) {
  const char* v = getenv(name);
  return (v && *v) ? atoi(v) : dflt;
}

Model::Model(const ifd_config& cfg) : cfg_(cfg) {
  build_plan();
  opt_stream_ = env_int("IFD_CONV_STREAM", 2);
  opt_x3_off_ = env_int("IFD_X3_OFF", 0);
  gn_fused_ = env_int("IFD_GN_FUSED", 1) != 0;
  opt_invariant_ = env_int("IFD_BATCH_INVARIANT", 0) != 0;
  opt_skip_sep_ = env_int("IFD_SKIP_SEP", 64);
}

int Model::set_option(const std::string& key, int v) {
  if (key == "conv_stream") {
    IFD_REQUIRE(v >= 0 && v <= 2, "conv_stream must be 0, 1 or 2");
    opt_stream_ = v;
  } else if (key == "x3_off") {
    opt_x3_off_ = v;
  } else if (key == "gn_fused") {
    gn_fused_ = v != 0;
  } else if (key == "skip_sep") {
    IFD_REQUIRE(v >= 0, "skip_sep must be >= 0");
    opt_skip_sep_ = v;
  } else if (key == "batch_invariant") {
    if ((v != 0) != (opt_invariant_ != 0)) ws_B_ = 0;  // split-K slab sizing depends on it: re-plan
    opt_invariant_ = v != 0;
  } else {
    IFD_REQUIRE(false, "unknown option " + key);
  }
  return 0;
}

int Model::get_option(const std::string& key, int* v) const {
  if (key == "conv_stream") *v = opt_stream_;
  else if (key == "x3_off") *v = opt_x3_off_;
  else if (key == "gn_fused") *v = gn_fused_ ? 1 : 0;
  else if (key == "batch_invariant") *v = opt_invariant_;
  else if (key == "skip_sep") *v = opt_skip_sep_;
  else IFD_REQUIRE(false, "unknown option " + key);
  return 0;
}

Model::~Model() {
  if (guard_) (void)hipFree(guard_);
  if (wblob_) (void)hipFree(wblob_);
  if (ws_) (void)hipFree(ws_);
  for (auto e : ev_pool_) (void)hipEventDestroy(e);
}

hipEvent_t Model::take_event() {
  if (ev_used_ == ev_pool_.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ev_pool_.push_back(e);
  }
  return ev_pool_[ev_used_++];
}

void Model::prof_begin(hipStream_t s, hipEvent_t* e0, const char* name) {
  *e0 = nullptr;
  if (!prof_on_) return;
  // name filter (profile_filter): record only the launches whose name starts with it, so a timed
  // region pays the event packets for the kernel it measures and not for every launch
  if (!prof_filter_.empty() && (!name || strncmp(name, prof_filter_.c_str(), prof_filter_.size()) != 0)) return;
  *e0 = take_event();
  if (*e0) (void)hipEventRecord(*e0, s);
}

void Model::prof_end(hipStream_t s, hipEvent_t e0, const std::string& name, double flops, double bytes) {
  if (!prof_on_ || !e0) return;
  hipEvent_t e1 = take_event();
  if (!e1) return;
  (void)hipEventRecord(e1, s);
  prof_.push_back({name, flops, bytes, e0, e1});
}

int Model::profile_filter(const char* prefix) {
  prof_filter_ = prefix ? prefix : "";
  return 0;
}

int Model::profile_enable(int on) {
  prof_on_ = on != 0;
  prof_layers_ = on == 2;
  prof_.clear();
  ev_used_ = 0;
  return 0;
}

// JSON: {"kernels": {name: {"count", "ms", "flops", "bytes"}}}; call after the stream is synchronised.
int Model::profile_report(std::string& json) {
  std::map<std::string, std::array<double, 4>> agg;
  for (auto& r : prof_) {
    float ms = 0.f;
    IFD_CHECK_HIP(hipEventElapsedTime(&ms, r.e0, r.e1));
    auto& a = agg[r.name];
    a[0] += 1;
    a[1] += ms;
    a[2] += r.flops;
    a[3] += r.bytes;
  }
  json = "{\"kernels\": {";
  bool first = true;
  for (auto& kv : agg) {
    char buf[512];
    snprintf(buf, sizeof(buf), "%s\"%s\": {\"count\": %.0f, \"ms\": %.6f, \"flops\": %.6e, \"bytes\": %.6e}",
             first ? "" : ", ", kv.first.c_str(), kv.second[0], kv.second[1], kv.second[2], kv.second[3]);
    json += buf;
    first = false;
  }
  json += "}}";
  prof_.clear();
  ev_used_ = 0;
  return 0;
}

void Model::add_param(const std::string& n, std::vector<int64_t> shape) { params_.push_back({n, std::move(shape)}); }

static ConvW make_conv(const std::string& w, const std::string& b, int cin, int cout, int taps) {
  ConvW c;
  c.cin = cin;
  c.cin_pad = ceil_to(cin, 8);
  c.cout = cout;
  c.bn = conv_pick_bn(cout, taps, 0, 0, 0);
  c.cout_pad = ceil_to(cout, c.bn);
  c.taps = taps;
  c.wname = w;
  c.bname = b;
  return c;
}

void Model::build_plan() {
  const int mc = cfg_.model_channels;
  emb_dim_ = 4 * mc;
  add_param("time_embed.0.weight", {emb_dim_, mc});
  add_param("time_embed.0.bias", {emb_dim_});
  add_param("time_embed.2.weight", {emb_dim_, emb_dim_});
  add_param("time_embed.2.bias", {emb_dim_});

  auto has_attn = [&](int ds) {
    for (int i = 0; i < cfg_.num_attention; ++i)
      if (cfg_.attention_ds[i] == ds) return true;
    return false;
  };
  auto add_res = [&](const std::string& p, int cin, int cout, int xf, int c_cat) {
    ResP r;
    r.prefix = p;
    r.cin = cin;
    r.cout = cout;
    r.xf = xf;
    r.c_cat = c_cat;
    r.gn1.C = cin;
    r.gn1.prefix = p + "in_layers.0.";
    r.conv1 = make_conv(p + "in_layers.2.weight", p + "in_layers.2.bias", cin, cout, 9);
    r.gn2.C = cout;
    r.gn2.prefix = p + "out_layers.0.";
    r.conv2 = make_conv(p + "out_layers.3.weight", p + "out_layers.3.bias", cout, cout, 9);
    add_param(p + "in_layers.0.weight", {cin});
    add_param(p + "in_layers.0.bias", {cin});
    add_param(p + "in_layers.2.weight", {cout, cin, 3, 3});
    add_param(p + "in_layers.2.bias", {cout});
    add_param(p + "emb_layers.1.weight", {2 * cout, emb_dim_});
    add_param(p + "emb_layers.1.bias", {2 * cout});
    add_param(p + "out_layers.0.weight", {cout});
    add_param(p + "out_layers.0.bias", {cout});
    add_param(p + "out_layers.3.weight", {cout, cout, 3, 3});
    add_param(p + "out_layers.3.bias", {cout});
    if (cin != cout) {
      add_param(p + "skip_connection.weight", {cout, cin, 1, 1});
      add_param(p + "skip_connection.bias", {cout});
      r.conv2.has_skip = true;
      r.conv2.cs = cin;
      r.conv2.cs_pad = ceil_to(cin, 8);
      r.conv2.swname = p + "skip_connection.weight";
      r.conv2.sbname = p + "skip_connection.bias";
    }
    r.emb_off = emb_total_;
    emb_total_ += 2 * cout;
    res_.push_back(r);
    return (int)res_.size() - 1;
  };
  auto add_attn = [&](const std::string& p, int c) {
    AttnP a;
    a.prefix = p;
    a.C = c;
    a.gn.C = c;
    a.gn.prefix = p + "norm.";
    a.qkv = make_conv(p + "qkv.weight", p + "qkv.bias", c, 3 * c, 1);
    a.proj = make_conv(p + "proj_out.weight", p + "proj_out.bias", c, c, 1);
    add_param(p + "norm.weight", {c});
    add_param(p + "norm.bias", {c});
    add_param(p + "qkv.weight", {3 * c, c, 1});
    add_param(p + "qkv.bias", {3 * c});
    add_param(p + "proj_out.weight", {c, c, 1});
    add_param(p + "proj_out.bias", {c});
    attn_.push_back(a);
    return (int)attn_.size() - 1;
  };

  int res = cfg_.image_size;
  int ch = cfg_.channel_mult[0] * mc;
  conv_in_ = make_conv("input_blocks.0.0.weight", "input_blocks.0.0.bias", 16, ch, 9);
  conv_in_.cin = cfg_.in_channels;  // packed input carries 16 channels, 9 real
  conv_in_.cin_pad = 16;
  add_param("input_blocks.0.0.weight", {ch, cfg_.in_channels, 3, 3});
  add_param("input_blocks.0.0.bias", {ch});
  in_blocks_.push_back({});
  in_ch_.push_back(ch);
  in_res_.push_back(res);
  int ds = 1;
  for (int level = 0; level < cfg_.num_levels; ++level) {
    const int mult = cfg_.channel_mult[level];
    for (int k = 0; k < cfg_.num_res_blocks; ++k) {
      const int i = (int)in_blocks_.size();
      const std::string p = "input_blocks." + std::to_string(i) + ".";
      const int out = mult * mc;
      std::vector<LayerP> L;
      L.push_back({L_RES, add_res(p + "0.", ch, out, XF_NONE, 0), res});
      ch = out;
      if (has_attn(ds)) L.push_back({L_ATTN, add_attn(p + "1.", ch), res});
      in_blocks_.push_back(L);
      in_ch_.push_back(ch);
      in_res_.push_back(res);
    }
    if (level != cfg_.num_levels - 1) {
      const int i = (int)in_blocks_.size();
      const std::string p = "input_blocks." + std::to_string(i) + ".";
      std::vector<LayerP> L;
      L.push_back({L_RES, add_res(p + "0.", ch, ch, XF_DOWN, 0), res});
      in_blocks_.push_back(L);
      ds *= 2;
      res /= 2;
      in_ch_.push_back(ch);
      in_res_.push_back(res);
    }
  }
  mid_.push_back({L_RES, add_res("middle_block.0.", ch, ch, XF_NONE, 0), res});
  mid_.push_back({L_ATTN, add_attn("middle_block.1.", ch), res});
  mid_.push_back({L_RES, add_res("middle_block.2.", ch, ch, XF_NONE, 0), res});
  std::vector<int> chans = in_ch_;
  int j = 0;
  for (int level = cfg_.num_levels - 1; level >= 0; --level) {
    const int mult = cfg_.channel_mult[level];
    for (int k = 0; k < cfg_.num_res_blocks + 1; ++k) {
      const int ich = chans.back();
      chans.pop_back();
      const std::string p = "output_blocks." + std::to_string(j) + ".";
      const int out = mc * mult;
      std::vector<LayerP> L;
      L.push_back({L_RES, add_res(p + "0.", ch + ich, out, XF_NONE, ich), res});
      ch = out;
      if (has_attn(ds)) L.push_back({L_ATTN, add_attn(p + "1.", ch), res});
      if (level && k == cfg_.num_res_blocks) {
        L.push_back({L_RES, add_res(p + std::to_string(L.size()) + ".", ch, ch, XF_UP, 0), res});
        ds /= 2;
        res *= 2;
      }
      out_blocks_.push_back(L);
      ++j;
    }
  }
  gn_out_.C = ch;
  gn_out_.prefix = "out.0.";
  add_param("out.0.weight", {ch});
  add_param("out.0.bias", {ch});
  conv_out_ = make_conv("out.2.weight", "out.2.bias", ch, cfg_.out_channels, 9);
  add_param("out.2.weight", {cfg_.out_channels, ch, 3, 3});
  add_param("out.2.bias", {cfg_.out_channels});
}

int Model::load(const std::string& name_in, const float* data, const int64_t* shape, int ndim) {
  std::string name = name_in;
  if (name.rfind("base_model.", 0) == 0) name = name.substr(11);
  const ParamSpec* spec = nullptr;
  for (auto& p : params_)
    if (p.name == name) spec = &p;
  IFD_REQUIRE(spec != nullptr, "unexpected parameter " + name_in);
  IFD_REQUIRE((int)spec->shape.size() == ndim, "rank mismatch for " + name);
  size_t numel = 1;
  for (int i = 0; i < ndim; ++i) {
    IFD_REQUIRE(spec->shape[i] == shape[i], "shape mismatch for " + name);
    numel *= (size_t)shape[i];
  }
  std::vector<float> buf(numel);
  IFD_CHECK_HIP(hipMemcpy(buf.data(), data, numel * sizeof(float), hipMemcpyDefault));
  host_[name] = std::move(buf);
  finalized_ = false;
  return 0;
}

// Packed conv weight layout: [Cout_pad/BN][Cin_pad/8][taps][q=2][BN][4], element
//   W[ct*BN + col][ch*8 + q*4 + j][tap/3][tap%3]  (zero outside [Cout) x [Cin)).
static void pack_conv(const std::vector<float>& w, int cout, int cin, int taps, int bn, int cin_pad, int cout_pad,
                      std::vector<float>& blob, size_t off) {
  const int nch = cin_pad / 8;
  for (int ct = 0; ct < cout_pad / bn; ++ct)
    for (int chk = 0; chk < nch; ++chk)
      for (int tap = 0; tap < taps; ++tap)
        for (int q = 0; q < 2; ++q)
          for (int col = 0; col < bn; ++col)
            for (int jj = 0; jj < 4; ++jj) {
              const int co = ct * bn + col, ci = chk * 8 + q * 4 + jj;
              float v = 0.f;
              if (co < cout && ci < cin) v = w[((size_t)co * cin + ci) * taps + tap];
              blob[off + ((((size_t)(ct * nch + chk) * taps + tap) * 2 + q) * bn + col) * 4 + jj] = v;
            }
}

// 3xf16 split packing: [Cout_pad/BN][Cin_pad/16][taps][part][h][BN][8] f16 (2 per float slot),
// element (part, h, col, j) of (ct, chunk, tap) = split part of W[ct*BN + col][chunk*16 + 8h + j][tap]:
// part 0 = f16(w) * 2^11 (exact), part 1 = f16((w - f16(w)) * 2^11) (conv_x3.hip). Returns false
// if a weight is outside the scaled part's f16 range (|w| >= 32), leaving the layer on fp32.
static bool pack_conv_x3(const std::vector<float>& w, int cout, int cin, int taps, int bn, int cin_pad16,
                         int cout_pad, std::vector<float>& blob, size_t off) {
  const int nch = cin_pad16 / 16;
  _Float16* dst = reinterpret_cast<_Float16*>(blob.data() + off);
  bool ok = true;
  for (int ct = 0; ct < cout_pad / bn; ++ct)
    for (int chk = 0; chk < nch; ++chk)
      for (int tap = 0; tap < taps; ++tap)
        for (int part = 0; part < 2; ++part)
          for (int hh = 0; hh < 2; ++hh)
            for (int col = 0; col < bn; ++col)
              for (int j = 0; j < 8; ++j) {
                const int co = ct * bn + col, ci = chk * 16 + hh * 8 + j;
                float v = 0.f;
                if (co < cout && ci < cin) v = w[((size_t)co * cin + ci) * taps + tap];
                const _Float16 hi = (_Float16)v;
                _Float16 o;
                if (part == 0) {
                  const float s = (float)hi * 2048.0f;
                  if (!(std::fabs(s) <= 65504.0f)) ok = false;
                  o = (_Float16)s;
                } else {
                  o = (_Float16)((v - (float)hi) * 2048.0f);
                }
                dst[((((((size_t)ct * nch + chk) * taps + tap) * 2 + part) * 2 + hh) * bn + col) * 8 + j] = o;
              }
  return ok;
}

// 3xf16 1x1 skip packing in kSkipChunk-channel chunks (conv_x3.hip skip_chunk): [Cout_pad/BN][Cs_pad/K][q]
// [part][h][BN][8] f16, element (q, part, h, col, j) of (ct, chunk s) = split part of
// W[ct*BN + col][K s + K/2 h + 8 q + j] (the consumer lane of channel half h holds channels K/2 h ..
// K/2 (h + 1) - 1 of the chunk; sub-chunk q of the k = 16 MFMA step takes 8 of them). Same parts and
// range check as pack_conv_x3.
static constexpr int kSkipChunk = 32;
static bool pack_skip_x3(const std::vector<float>& w, int cout, int cin, int bn, int cs_pad, int cout_pad,
                         std::vector<float>& blob, size_t off) {
  constexpr int K = kSkipChunk, NQ = K / 16;
  const int ns = cs_pad / K;
  _Float16* dst = reinterpret_cast<_Float16*>(blob.data() + off);
  bool ok = true;
  for (int ct = 0; ct < cout_pad / bn; ++ct)
    for (int sk = 0; sk < ns; ++sk)
      for (int q = 0; q < NQ; ++q)
        for (int part = 0; part < 2; ++part)
          for (int hh = 0; hh < 2; ++hh)
            for (int col = 0; col < bn; ++col)
              for (int j = 0; j < 8; ++j) {
                const int co = ct * bn + col, ci = sk * K + hh * (K / 2) + q * 8 + j;
                const float v = (co < cout && ci < cin) ? w[(size_t)co * cin + ci] : 0.f;
                const _Float16 hi = (_Float16)v;
                _Float16 o;
                if (part == 0) {
                  const float sc = (float)hi * 2048.0f;
                  if (!(std::fabs(sc) <= 65504.0f)) ok = false;
                  o = (_Float16)sc;
                } else {
                  o = (_Float16)((v - (float)hi) * 2048.0f);
                }
                dst[((((((size_t)ct * ns + sk) * NQ + q) * 2 + part) * 2 + hh) * bn + col) * 8 + j] = o;
              }
  return ok;
}

// Split packing of a skip_connection for skip_x3.hip: [cout/ntc][K/16][part][h][ntc][8] f16, element
// (part, h, col, j) of (tile nt, step ks) = split part of Ws[nt*ntc + col][16 ks + 8 h + j] (the MFMA
// B operand of lane (h, col)). Same parts and range check as pack_conv_x3.
static bool pack_skip1x1_x3(const std::vector<float>& w, int cout, int cin, int ntc, int cs_pad,
                            std::vector<float>& blob, size_t off) {
  const int ks_n = cs_pad / 16;
  _Float16* dst = reinterpret_cast<_Float16*>(blob.data() + off);
  bool ok = true;
  for (int nt = 0; nt < cout / ntc; ++nt)
    for (int ks = 0; ks < ks_n; ++ks)
      for (int part = 0; part < 2; ++part)
        for (int hh = 0; hh < 2; ++hh)
          for (int col = 0; col < ntc; ++col)
            for (int j = 0; j < 8; ++j) {
              const int co = nt * ntc + col, ci = ks * 16 + hh * 8 + j;
              const float v = ci < cin ? w[(size_t)co * cin + ci] : 0.f;
              const _Float16 hi = (_Float16)v;
              _Float16 o;
              if (part == 0) {
                const float sc = (float)hi * 2048.0f;
                if (!(std::fabs(sc) <= 65504.0f)) ok = false;
                o = (_Float16)sc;
              } else {
                o = (_Float16)((v - (float)hi) * 2048.0f);
              }
              dst[(((((size_t)nt * ks_n + ks) * 2 + part) * 2 + hh) * ntc + col) * 8 + j] = o;
            }
  return ok;
}

// K chunks of a conv on the split kernel: 16-channel 3x3 chunks + kSkipChunk-channel 1x1 skip chunks; a
// plain 1x1 conv (attention qkv / proj_out) runs as skip chunks only
static int x3_nchunks(const ConvW& cw) {
  if (cw.taps == 1 && !cw.has_skip) return cw.cin_pad / kSkipChunk;
  return cw.cin_pad / 16 + (cw.has_skip ? cw.cs_pad / kSkipChunk : 0);
}

int Model::guard_reset(hipStream_t s) {
  if (!guard_) {
    IFD_CHECK_HIP(hipMalloc(&guard_, 64));
    IFD_CHECK_HIP(hipMemset(guard_, 0, 64));
  }
  IFD_CHECK_HIP(hipMemsetAsync(guard_, 0, sizeof(unsigned), s));
  return 0;
}

int Model::guard_read(hipStream_t s, int* tripped) {
  *tripped = 0;
  if (!guard_) return 0;
  unsigned v = 0;
  IFD_CHECK_HIP(hipMemcpyAsync(&v, guard_, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  IFD_CHECK_HIP(hipStreamSynchronize(s));
  *tripped = v != 0;
  return 0;
}

int Model::guard_copy_async(hipStream_t s, unsigned* host_dst) {
  if (!guard_) {
    IFD_CHECK_HIP(hipMalloc(&guard_, 64));
    IFD_CHECK_HIP(hipMemset(guard_, 0, 64));
  }
  IFD_CHECK_HIP(hipMemcpyAsync(host_dst, guard_, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  return 0;
}

int Model::set_precision(int prec) {
  IFD_REQUIRE(prec == IFD_PREC_FP32 || prec == IFD_PREC_3XF16 || prec == IFD_PREC_F16, "unknown precision mode");
  prec_ = prec;
  return 0;
}

int Model::finalize() {
  for (auto& p : params_) IFD_REQUIRE(host_.count(p.name), "missing parameter " + p.name);
  // size the blob
  size_t n = 0;
  auto reserve = [&](size_t cnt) {
    size_t o = n;
    n += (cnt + 3) / 4 * 4;  // keep 16-byte alignment
    return o;
  };
  auto plan_conv = [&](ConvW& c) {
    c.w_off = reserve((size_t)c.cout_pad * c.cin_pad * c.taps);
    c.b_off = reserve(c.cout_pad);
    if (c.has_skip) c.ws_off = reserve((size_t)c.cout_pad * c.cs_pad);
    // 3xf16 packing (two f16 parts = one float slot per weight) for the layers conv_x3 can run
    c.x3_off = c.x3s_off = 0;
    if (c.taps == 9 && c.bn == 64 && c.cin_pad % 16 == 0 && (!c.has_skip || c.cs_pad % kSkipChunk == 0)) {
      c.x3_off = reserve((size_t)c.cout_pad * c.cin_pad * c.taps);
      if (c.has_skip) c.x3s_off = reserve((size_t)c.cout_pad * c.cs_pad);
    } else if (c.taps == 1 && c.bn == 64 && c.cin_pad % kSkipChunk == 0 && !c.has_skip) {
      c.x3s_off = reserve((size_t)c.cout_pad * c.cin_pad);  // a 1x1 conv runs as 1x1 chunks only
    }
    c.sk_off = c.bmain_off = c.sbias_off = 0;
    c.sk_ntc = 0;
    if (c.has_skip && c.x3_off && c.cout == c.cout_pad) c.sk_ntc = skip_x3_ntc(c.cs_pad, c.cout);
    if (c.sk_ntc) {
      c.sk_off = reserve((size_t)c.cout * c.cs_pad);
      c.bmain_off = reserve(c.cout_pad);
      c.sbias_off = reserve(c.cout_pad);
    }
  };
  auto plan_gn = [&](GNW& g) {
    g.g_off = reserve(g.C);
    g.b_off = reserve(g.C);
  };
  const int mc = cfg_.model_channels;
  te_w0_ = reserve((size_t)mc * emb_dim_);
  te_b0_ = reserve(emb_dim_);
  te_w2_ = reserve((size_t)emb_dim_ * emb_dim_);
  te_b2_ = reserve(emb_dim_);
  freqs_ = reserve(mc / 2);
  embw_ = reserve((size_t)emb_dim_ * emb_total_);
  embb_ = reserve(emb_total_);
  plan_conv(conv_in_);
  for (auto& r : res_) {
    plan_gn(r.gn1);
    plan_conv(r.conv1);
    plan_gn(r.gn2);
    plan_conv(r.conv2);
  }
  for (auto& a : attn_) {
    plan_gn(a.gn);
    plan_conv(a.qkv);
    plan_conv(a.proj);
  }
  plan_gn(gn_out_);
  plan_conv(conv_out_);
  conv_out_.head_off = 0;
  if (conv_out_.taps == 9 && conv_out_.cin % 16 == 0 && (conv_out_.cout == 6 || conv_out_.cout == 3))
    conv_out_.head_off = reserve(conv_head_pack_floats(conv_out_.cin));
  conv_out_.head_x3_off = 0;
  if (conv_out_.head_off && conv_out_.cin % 32 == 0 && conv_out_.cin <= 128)
    conv_out_.head_x3_off = reserve(conv_head_x3_pack_floats(conv_out_.cin));

  std::vector<float> blob(n, 0.f);
  auto put = [&](size_t off, const std::vector<float>& v) { std::copy(v.begin(), v.end(), blob.begin() + off); };
  auto fill_conv = [&](ConvW& c) {
    pack_conv(host_[c.wname], c.cout, c.cin, c.taps, c.bn, c.cin_pad, c.cout_pad, blob, c.w_off);
    c.x3_ok = c.x3_off && pack_conv_x3(host_[c.wname], c.cout, c.cin, c.taps, c.bn, c.cin_pad, c.cout_pad, blob,
                                       c.x3_off);
    if (c.taps == 1 && c.x3s_off)
      c.x3_ok = pack_skip_x3(host_[c.wname], c.cout, c.cin, c.bn, c.cin_pad, c.cout_pad, blob, c.x3s_off);
    if (c.x3_ok && c.has_skip)
      c.x3_ok = pack_skip_x3(host_[c.swname], c.cout, c.cs, c.bn, c.cs_pad, c.cout_pad, blob, c.x3s_off);
    const auto& b = host_[c.bname];
    for (int i = 0; i < c.cout; ++i) blob[c.b_off + i] = b[i];
    if (c.has_skip) {
      pack_conv(host_[c.swname], c.cout, c.cs, 1, c.bn, c.cs_pad, c.cout_pad, blob, c.ws_off);
      const auto& sb = host_[c.sbname];
      // bias of h (conv) and of skip_connection(x) are both added once per output element
      for (int i = 0; i < c.cout; ++i) blob[c.b_off + i] = b[i] + sb[i];
    }
    c.sk_ok = false;
    if (c.sk_ntc) {
      c.sk_ok = c.x3_ok && pack_skip1x1_x3(host_[c.swname], c.cout, c.cs, c.sk_ntc, c.cs_pad, blob, c.sk_off);
      const auto& sb = host_[c.sbname];
      for (int i = 0; i < c.cout; ++i) {
        blob[c.bmain_off + i] = b[i];
        blob[c.sbias_off + i] = sb[i];
      }
    }
  };
  auto fill_gn = [&](GNW& g) {
    put(g.g_off, host_[g.prefix + "weight"]);
    put(g.b_off, host_[g.prefix + "bias"]);
  };
  // time embedding: transpose [out][in] -> [in][out]
  {
    const auto& w0 = host_["time_embed.0.weight"];
    for (int o = 0; o < emb_dim_; ++o)
      for (int i = 0; i < mc; ++i) blob[te_w0_ + (size_t)i * emb_dim_ + o] = w0[(size_t)o * mc + i];
    put(te_b0_, host_["time_embed.0.bias"]);
    const auto& w2 = host_["time_embed.2.weight"];
    for (int o = 0; o < emb_dim_; ++o)
      for (int i = 0; i < emb_dim_; ++i) blob[te_w2_ + (size_t)i * emb_dim_ + o] = w2[(size_t)o * emb_dim_ + i];
    put(te_b2_, host_["time_embed.2.bias"]);
    // freqs = exp(-ln(10000) * arange(half, fp32) / half) in fp32, as code/nn.py:54-56
    const int half = mc / 2;
    const float c = (float)(-std::log(10000.0));
    for (int i = 0; i < half; ++i) {
      volatile float prod = c * (float)i;
      volatile float q = prod / (float)half;
      blob[freqs_ + i] = std::exp(q);
    }
  }
  for (auto& r : res_) {
    const auto& w = host_[r.prefix + "emb_layers.1.weight"];
    const auto& b = host_[r.prefix + "emb_layers.1.bias"];
    for (int o = 0; o < 2 * r.cout; ++o) {
      for (int i = 0; i < emb_dim_; ++i)
        blob[embw_ + (size_t)i * emb_total_ + r.emb_off + o] = w[(size_t)o * emb_dim_ + i];
      blob[embb_ + r.emb_off + o] = b[o];
    }
  }
  fill_conv(conv_in_);
  for (auto& r : res_) {
    fill_gn(r.gn1);
    fill_conv(r.conv1);
    fill_gn(r.gn2);
    fill_conv(r.conv2);
    r.conv2_res = r.conv2;
    if (r.conv2.sk_ok) {  // the same conv without its 1x1 segment, own bias only
      ConvW& c = r.conv2_res;
      c.has_skip = false;
      c.cs = c.cs_pad = 0;
      c.ws_off = c.x3s_off = 0;
      c.b_off = c.bmain_off;
      c.sk_ok = false;
    }
  }
  for (auto& a : attn_) {
    fill_gn(a.gn);
    fill_conv(a.qkv);
    fill_conv(a.proj);
  }
  fill_gn(gn_out_);
  fill_conv(conv_out_);
  if (conv_out_.head_off)
    conv_head_pack(host_[conv_out_.wname].data(), conv_out_.cout, conv_out_.cin, blob.data() + conv_out_.head_off);
  conv_out_.head_x3_ok = conv_out_.head_x3_off &&
                         conv_head_x3_pack(host_[conv_out_.wname].data(), conv_out_.cout, conv_out_.cin,
                                           blob.data() + conv_out_.head_x3_off);

  if (wblob_) IFD_CHECK_HIP(hipFree(wblob_));
  wblob_ = nullptr;
  IFD_CHECK_HIP(hipMalloc(&wblob_, n * sizeof(float)));
  IFD_CHECK_HIP(hipMemcpy(wblob_, blob.data(), n * sizeof(float), hipMemcpyHostToDevice));
  wblob_floats_ = n;
  finalized_ = true;
  return 0;
}

// Workspace arena plan at batch B (host arithmetic only, no device calls): float offsets of every
// area, and the (activation buffer, granule-statistics area) pairs. Returns the arena size in floats.
size_t Model::plan_workspace(int B, WsLayout& w, std::vector<std::pair<size_t, size_t>>& stat_of) const {
  const int R = cfg_.image_size;
  size_t n = 0;
  auto reserve = [&](size_t cnt) {
    size_t o = n;
    n += (cnt + 63) / 64 * 64;
    return o;
  };
  size_t maxact = 0, maxqkv = 1, maxC = 16;
  w.o_hs_.clear();
  for (size_t i = 0; i < in_ch_.size(); ++i) {
    const size_t sz = (size_t)B * in_res_[i] * in_res_[i] * in_ch_[i];
    w.o_hs_.push_back(reserve(sz));
    maxact = std::max(maxact, sz);
  }
  for (auto& r : res_) {
    maxC = std::max<size_t>(maxC, std::max(r.cin, r.cout));
  }
  // worst activation size over all layers: every layer output is B * res^2 * C with res <= R
  for (auto& blk : out_blocks_)
    for (auto& L : blk) {
      int C = L.kind == L_RES ? res_[L.idx].cout : attn_[L.idx].C;
      int rr = L.res_in * ((L.kind == L_RES && res_[L.idx].xf == XF_UP) ? 2 : 1);
      maxact = std::max(maxact, (size_t)B * rr * rr * C);
    }
  for (auto& L : mid_) {
    int C = L.kind == L_RES ? res_[L.idx].cout : attn_[L.idx].C;
    maxact = std::max(maxact, (size_t)B * L.res_in * L.res_in * C);
  }
  for (auto& a : attn_) (void)a;
  for (size_t i = 0; i < in_blocks_.size(); ++i)
    for (auto& L : in_blocks_[i])
      if (L.kind == L_ATTN) maxqkv = std::max(maxqkv, (size_t)B * L.res_in * L.res_in * attn_[L.idx].C * 3);
  for (auto& blk : out_blocks_)
    for (auto& L : blk)
      if (L.kind == L_ATTN) maxqkv = std::max(maxqkv, (size_t)B * L.res_in * L.res_in * attn_[L.idx].C * 3);
  for (auto& L : mid_)
    if (L.kind == L_ATTN) maxqkv = std::max(maxqkv, (size_t)B * L.res_in * L.res_in * attn_[L.idx].C * 3);
  w.o_x0_ = reserve((size_t)B * R * R * 16);
  for (int k = 0; k < 3; ++k) w.o_bufs_[k] = reserve(maxact);
  w.o_t1_ = reserve(maxact);
  w.o_qkv_ = reserve(maxqkv);
  w.o_ao_ = reserve(maxqkv / 3 + 1);
  w.o_A_ = reserve((size_t)B * maxC);
  w.o_B_ = reserve((size_t)B * maxC);
  int slice;
  const int nsl = gn_slices(R * R, &slice);
  w.o_part_ = reserve((size_t)B * nsl * 32 * 3);
  // split-K slabs: worst case over every conv of the plan at this batch
  w.split_floats_ = 0;
  auto consider = [&](const ConvW& cw, int H) {
    for (int x3 = 0; x3 < 2; ++x3) {  // fp32 kernels' geometry and the split kernel's
      ConvParams g;
      std::memset(&g, 0, sizeof(g));
      fill_opts(g);
      g.cout_pad = cw.cout_pad;
      const int nch = x3 ? x3_nchunks(cw) : cw.cin_pad / 8;
      conv_geometry(g, H, H, B, cw.bn, nch, x3 == 1);
      if (x3 && cw.taps == 1 && !cw.has_skip && g.ksplit == 1 && nch % 2 == 0) g.ksplit = 2;  // see run_conv
      if (g.ksplit > 1) w.split_floats_ = std::max(w.split_floats_, (size_t)g.ksplit * B * H * H * cw.cout);
    }
  };
  // only the (conv, output resolution) pairs the plan runs: every layer knows its input resolution
  auto consider_layer = [&](const LayerP& L) {
    if (L.kind == L_RES) {
      const ResP& r = res_[L.idx];
      const int H = r.xf == XF_UP ? 2 * L.res_in : (r.xf == XF_DOWN ? L.res_in / 2 : L.res_in);
      consider(r.conv1, H);
      consider(r.conv2, H);
      if (r.conv2.sk_ok) consider(r.conv2_res, H);  // (the separate-skip plan's conv2)
    } else {
      consider(attn_[L.idx].qkv, L.res_in);
      consider(attn_[L.idx].proj, L.res_in);
    }
  };
  for (auto* blocks : {&in_blocks_, &out_blocks_})
    for (auto& blk : *blocks)
      for (auto& L : blk) consider_layer(L);
  for (auto& L : mid_) consider_layer(L);
  consider(conv_in_, R);
  w.o_split_ = reserve(std::max<size_t>(w.split_floats_, 64));
  // act+pool staging of the down-ResBlocks (3xf16 mode): B x (res/2)^2 x cin, worst over the plan
  size_t maxpool = 64;
  for (auto& blk : in_blocks_)
    for (auto& L : blk)
      if (L.kind == L_RES && res_[L.idx].xf == XF_DOWN)
        maxpool = std::max(maxpool, (size_t)B * (L.res_in / 2) * (L.res_in / 2) * res_[L.idx].cin);
  // ... and act(GN(x)) of the attention blocks' qkv conv (B x res^2 x C)
  for (auto* blocks : {&in_blocks_, &out_blocks_})
    for (auto& blk : *blocks)
      for (auto& L : blk)
        if (L.kind == L_ATTN) maxpool = std::max(maxpool, (size_t)B * L.res_in * L.res_in * attn_[L.idx].C);
  for (auto& L : mid_)
    if (L.kind == L_ATTN) maxpool = std::max(maxpool, (size_t)B * L.res_in * L.res_in * attn_[L.idx].C);
  w.pool_floats_ = maxpool;
  w.o_pool_ = reserve(maxpool);
  w.o_pool2_ = reserve(maxpool);  // pooled residual (a down-ResBlock keeps cin == cout)
  w.o_emb_ = reserve((size_t)B * emb_dim_);
  w.o_h1_ = reserve((size_t)B * emb_dim_);
  w.o_E_ = reserve((size_t)B * emb_total_);
  // granule statistics areas: a tensor at resolution r with C channels has at most
  // max(r^2/64, 1) entries of C/4 (mean, M2) pairs per image
  auto stat_floats = [&](int r, int C) { return (size_t)B * std::max(r * r / 64, 1) * (C / 4) * 2; };
  stat_of.clear();  // (buffer offset, stat offset)
  for (size_t i = 0; i < w.o_hs_.size(); ++i) stat_of.push_back({w.o_hs_[i], reserve(stat_floats(in_res_[i], in_ch_[i]))});
  size_t worst = 0;
  for (int r = 1; r <= R; r *= 2) worst = std::max(worst, stat_floats(r, (int)std::min<size_t>(maxC, 512)));
  worst = std::max(worst, stat_floats(R, 512));
  for (int k = 0; k < 3; ++k) stat_of.push_back({w.o_bufs_[k], reserve(worst)});
  stat_of.push_back({w.o_t1_, reserve(worst)});
  return n;
}

int64_t Model::workspace_bytes_for(int B) const {
  WsLayout w;
  std::vector<std::pair<size_t, size_t>> stat_of;
  return (int64_t)plan_workspace(B, w, stat_of) * 4;
}

int Model::ensure_workspace(int B) {
  if (ws_ && B <= ws_B_) return 0;
  WsLayout w;
  std::vector<std::pair<size_t, size_t>> stat_of;
  const size_t n = plan_workspace(B, w, stat_of);
  if (ws_) IFD_CHECK_HIP(hipFree(ws_));
  ws_ = nullptr;
  IFD_CHECK_HIP(hipMalloc(&ws_, n * sizeof(float)));
  ws_floats_ = n;
  ws_B_ = B;
  ly_ = w;
  stat_area_.clear();
  for (auto& so : stat_of) stat_area_[ws_ + so.first] = ws_ + so.second;
  return 0;
}

int Model::run_conv(const ConvW& cw, const float* in0, int c0, const float* in1, int c1, int N, int Hin, int H,
                    int xf, int act, const float* A, const float* Bc, const float* s0, int sc0, const float* s1,
                    int sc1, const float* res, int res_xf, int resH, float* out, int epi, hipStream_t s,
                    const StepCoeffs* sc, float* img, const float* gt, const float* mask, const float* noise,
                    const float* known) {
  ConvParams p;
  std::memset(&p, 0, sizeof(p));
  fill_opts(p);
  p.guard = guard_;
  p.x3_nprod = prec_ == IFD_PREC_F16 ? 1 : 3;
  const bool split_ = prec_ == IFD_PREC_3XF16 || prec_ == IFD_PREC_F16;  // the split-kernel modes
  p.in0 = in0; p.c0 = c0; p.in1 = in1; p.c1 = c1;
  p.N = N; p.Hin = Hin; p.Win = Hin; p.H = H; p.W = H;
  p.act = act; p.actA = A; p.actB = Bc;
  p.wpack = wblob_ + cw.w_off;
  p.bias = wblob_ + cw.b_off;
  p.cin_pad = cw.cin_pad; p.cout = cw.cout; p.cout_pad = cw.cout_pad;
  if (cw.has_skip) {
    p.s0 = s0; p.sc0 = sc0; p.s1 = s1; p.sc1 = sc1;
    p.wskip = wblob_ + cw.ws_off;
    p.cs_pad = cw.cs_pad;
  }
  p.res = res; p.res_xform = res_xf; p.res_H = resH; p.res_W = resH;
  p.out = out;
  p.epi = epi;
  IFD_REQUIRE((H & (H - 1)) == 0, "spatial size must be a power of two");
  // the persistent split kernel: 256-pixel tiles, K split over units at low resolution
  const bool x3_geo = split_ && cw.x3_ok && epi == EPI_NHWC;
  const int x3_chunks = x3_nchunks(cw);
  conv_geometry(p, H, H, N, cw.bn, x3_geo ? x3_chunks : cw.cin_pad / 8, x3_geo);
  if (epi != EPI_NHWC) p.ksplit = 1;
  p.part = ws_ + ly_.o_split_;
  IFD_REQUIRE(p.ksplit == 1 || (size_t)p.ksplit * N * H * H * cw.cout <= ly_.split_floats_, "split-K workspace");
  if (sc) p.sc = *sc;
  p.img = img; p.gt = gt; p.mask = mask; p.noise = noise; p.known = known;
  IFD_REQUIRE(c0 % 8 == 0 && c1 % 8 == 0 && c0 + c1 == cw.cin_pad, "conv input channels");
  IFD_REQUIRE(!cw.has_skip || (sc0 + sc1 == cw.cs_pad && sc0 % 8 == 0 && sc1 % 8 == 0), "skip channels");
  // option conv_stream selects the wide-layer kernel: 0 one tile per workgroup (conv.hip), 1 one
  // persistent workgroup per CU, 2 two persistent workgroups per CU (conv_stream.hip). The
  // batch-invariant geometry keeps the one-tile kernel: the stream kernels' eligibility depends on
  // the batch's tile count.
  const int stream_mode = opt_invariant_ ? 0 : opt_stream_;
  // 3xf16 1x1 conv (attention qkv / proj_out): the split kernel's 1x1 chunks over the raw operand,
  // act(GN(x)) materialised first when the conv has a prologue (act_apply, the conv prologue's
  // fp32 arithmetic)
  // development option x3_off (bisecting): 1 no 16x16 tiles, 2 no split-K, 4 no skip layers,
  // 8 no 8x8 four-image tiles, 16 no 1x1-only launches, 32 no split-MFMA output head
  const int x3_off = opt_x3_off_;
  auto x3_masked_for = [&](const ConvParams& g) {
    return ((x3_off & 1) && g.TW == 16) || ((x3_off & 2) && g.ksplit > 1) || ((x3_off & 4) && cw.has_skip) ||
           ((x3_off & 8) && g.TW == 8) || ((x3_off & 16) && cw.taps == 1);
  };
  if (split_ && cw.taps == 1 && cw.x3_ok && cw.x3s_off && epi == EPI_NHWC && !in1 &&
      xf == XF_NONE && !x3_masked_for(p)) {
    ConvParams q = p;
    q.in0 = nullptr; q.c0 = 0; q.in1 = nullptr; q.c1 = 0; q.cin_pad = 0; q.act = ACT_NONE;
    q.s0 = act != ACT_NONE ? ws_ + ly_.o_pool_ : in0; q.sc0 = c0; q.s1 = nullptr; q.sc1 = 0;
    q.wskip = wblob_ + cw.x3s_off; q.cs_pad = cw.cin_pad;
    // a residual (proj_out) is added by the split-K reduction: the split kernel's 1x1 path has none
    if (q.res && q.ksplit == 1 && x3_chunks % 2 == 0 && 2 * (size_t)N * H * H * cw.cout <= ly_.split_floats_) q.ksplit = 2;
    if (conv_x3_eligible(q, 1, XF_NONE, cw.bn)) {
      if (act != ACT_NONE) {
        IFD_REQUIRE((size_t)N * H * H * c0 <= ly_.pool_floats_, "act_apply workspace");
        hipEvent_t pe;
        prof_begin(s, &pe, "act_pool");
        const int e = launch_act_apply(in0, c0, N, H * H, act, A, Bc, ws_ + ly_.o_pool_, s);
        prof_end(s, pe, "act_pool", 0.0, 8.0 * N * (double)H * H * c0);
        IFD_LAUNCH_OK(e, "act_apply");
      }
      p = q;
      act = ACT_NONE;
    }
  }
  // 3xf16: the split kernel has no avg-pool prologue or residual; a down-ResBlock's convs read
  // act+pool(x) / pool(x) materialised by act_pool at the output resolution instead (the same
  // fp32 arithmetic as conv.hip's XF_DOWN paths)
  // ly_.o_pool2_ holds pool(in0) only for the conv that directly follows the act_pool that wrote it
  // (conv2 of the same down-ResBlock); any other conv in between invalidates it
  const float* pooled_prev = pooled_raw_;
  pooled_raw_ = nullptr;
  if (split_ && cw.x3_ok) {
    const bool pool_in = xf == XF_DOWN && !in1;
    const bool pool_res = res && res_xf == XF_DOWN;
    ConvParams q = p;
    if (pool_in) {
      q.in0 = ws_ + ly_.o_pool_;
      q.Hin = q.Win = H;
      q.act = ACT_NONE;
    }
    if (pool_res) {
      q.res = ws_ + ly_.o_pool2_;
      q.res_xform = XF_NONE;
      q.res_H = q.res_W = H;
    }
    if ((pool_in || pool_res) && conv_x3_eligible(q, cw.taps, pool_in ? (int)XF_NONE : xf, cw.bn)) {
      hipEvent_t pe;
      prof_begin(s, &pe, "act_pool");
      int e = 0;
      // conv1 of a down-ResBlock also pools its raw input for conv2's residual (same tensor, read
      // once); conv2 then finds pool(res) already in ly_.o_pool2_
      if (pool_in) {
        const bool raw_too = c0 == cw.cout;  // a down-ResBlock keeps its width: conv2's residual is in0
        e = launch_act_pool(in0, c0, N, Hin, act, A, Bc, ws_ + ly_.o_pool_, raw_too ? ws_ + ly_.o_pool2_ : nullptr, s);
        pooled_raw_ = raw_too ? in0 : nullptr;
      }
      if (!e && pool_res && res != pooled_prev)
        e = launch_act_pool(res, cw.cout, N, resH, ACT_NONE, nullptr, nullptr, ws_ + ly_.o_pool2_, nullptr, s);
      prof_end(s, pe, "act_pool", 0.0, 4.0 * N * (double)Hin * Hin * (c0 + (pool_res ? cw.cout : 0)) * 1.25);
      IFD_LAUNCH_OK(e, "act_pool");
      p = q;
      if (pool_in) {
        xf = XF_NONE;
        act = ACT_NONE;
      }
    }
  }
  const bool x3_masked = x3_masked_for(p);
  const bool use_x3 = split_ && cw.x3_ok && !x3_masked && conv_x3_eligible(p, cw.taps, xf, cw.bn);
  IFD_REQUIRE(use_x3 || p.cin_pad == cw.cin_pad, "1x1-only operand rewrite without the split kernel");
  if (use_x3) {
    p.wpack = wblob_ + cw.x3_off;
    if (cw.has_skip) p.wskip = wblob_ + cw.x3s_off;
  } else if (x3_geo) {  // not split-eligible after all: the fp32 kernels' own geometry
    conv_geometry(p, H, H, N, cw.bn, cw.cin_pad / 8);
  }
  // the output head (cout 6): fp32 VALU kernel, or in the split modes (3xf16, f16) the split-MFMA head
  const bool use_head = !use_x3 && cw.head_off && conv_head_eligible(p, cw.taps, xf);
  const bool use_head_x3 = use_head && split_ && cw.head_x3_ok && !(opt_x3_off_ & 32) &&
                           conv_head_x3_eligible(p, cw.taps, xf);
  const bool use_stream = !use_head && (use_x3 || (stream_mode != 0 && conv_stream_eligible(p, cw.taps, xf, cw.bn)));
  // fused GroupNorm statistics of the output (single-image tiles, no split-K; not mode 1)
  p.gstat = nullptr;
  p.gstat_E = 0;
  if (gn_fused_ && epi == EPI_NHWC && p.ksplit == 1 && p.IMGS == 1 && cw.bn == 64 &&
      (!use_stream || use_x3 || stream_mode == 2)) {
    auto it = stat_area_.find(out);
    if (it != stat_area_.end()) {
      p.gstat = it->second;
      p.gstat_E = p.tiles_x * p.tiles_y * (use_stream ? 4 : 1);
    }
  }
#if IFD_TRACE
  // development builds: dump per-block timestamps of the IFD_TRACE_NTH launch whose layer name
  // contains IFD_TRACE_MATCH into IFD_TRACE_FILE (+ ".json" with the geometry)
  const char* tmatch = getenv("IFD_TRACE_MATCH");  // read per call: a driver may set it mid-run
  const int tnth = getenv("IFD_TRACE_NTH") ? atoi(getenv("IFD_TRACE_NTH")) : 0;
  static int tseen = 0;
  static std::string tlast;
  if (tmatch && tlast != tmatch) {
    tlast = tmatch;
    tseen = 0;
  }
  unsigned long long* tbuf = nullptr;
  size_t tblocks = 0;
  char tname[160];
  snprintf(tname, sizeof(tname), "r%d %d+%d->%d skip%d xf%d", H, c0, c1, cw.cout, cw.has_skip ? cw.cs : 0, xf);
  if (tmatch && strstr(tname, tmatch) && tseen++ == tnth) {
    tblocks = (size_t)((p.npix_tiles + 7) / 8 * 8) * (cw.cout_pad / cw.bn) * p.ksplit;
    IFD_CHECK_HIP(hipMalloc(&tbuf, tblocks * 64 * sizeof(unsigned long long)));
    IFD_CHECK_HIP(hipMemsetAsync(tbuf, 0, tblocks * 64 * sizeof(unsigned long long), s));
    p.trace = tbuf;
  }
#endif
  char nm[160] = "";
  double flops = 0.0, bytes = 0.0;
  if (prof_on_) {
    // algorithmic work: 2*MAC over real channels; bytes = activations in + weights + out (once each)
    const int cin_real = (&cw == &conv_in_) ? cfg_.in_channels : cw.cin;
    const double pix = (double)N * H * H;
    flops = 2.0 * pix * cw.cout * ((double)cw.taps * cin_real + (cw.has_skip ? cw.cs : 0));
    bytes = 4.0 * ((double)N * Hin * Hin * (c0 + c1) + pix * cw.cout + (double)cw.cout * cw.cin * cw.taps +
                   (cw.has_skip ? pix * cw.cs : 0) + (res ? pix * cw.cout : 0));
    if (prof_layers_)
      snprintf(nm, sizeof(nm), "%s<%d,%d,%d,%d> r%d %d+%d->%d skip%d",
               use_x3 ? "conv_x3" : (use_head ? "conv_head" : (use_stream ? "conv_stream" : "conv_kernel")), p.bm,
               cw.bn, cw.taps, xf, H, c0, c1, cw.cout, cw.has_skip ? cw.cs : 0);
    else if (use_x3)
      snprintf(nm, sizeof(nm), "conv_x3_kernel<%d,%s,%d,%d>", xf, cw.has_skip ? "true" : "false", p.TW, p.x3_nprod);
    else if (use_head_x3)
      snprintf(nm, sizeof(nm), "conv_head_x3_kernel<%d>", cw.cout);
    else if (use_head)
      snprintf(nm, sizeof(nm), "conv_head_kernel<%d>", cw.cout);
    else if (use_stream && stream_mode == 2)  // template arguments as in the rocprof kernel name
      snprintf(nm, sizeof(nm), "conv_stream2_kernel<%d>", xf);
    else if (use_stream)
      snprintf(nm, sizeof(nm), "conv_stream_kernel<%d,8>", xf);
    else  // (BM,BN,WGM,WGN,TAPS,XF)
      snprintf(nm, sizeof(nm), "conv_kernel<%d,%d,%s,%d,%d>", p.bm, cw.bn,
               (p.bm == 256 || cw.bn == 32) ? "4,1" : "2,2", cw.taps, xf);
  }
  hipEvent_t e0;
  prof_begin(s, &e0, nm);
  if (use_head) p.ksplit = 1;
  int e = use_x3       ? launch_conv_x3(p, xf, s)
          : use_head_x3 ? launch_conv_head_x3(p, wblob_ + cw.head_x3_off, s)
          : use_head   ? launch_conv_head(p, wblob_ + cw.head_off, s)
          : use_stream ? launch_conv_stream(p, xf, stream_mode, s)
                       : launch_conv(p, cw.taps, xf, cw.bn, s);
  if (p.gstat)
    stat_[out] = StatRec{p.gstat, p.gstat_E, 4.0f * (use_stream ? 64 : p.bm), cw.cout};
  else
    stat_.erase(out);
#if IFD_TRACE
  if (tbuf) {
    IFD_CHECK_HIP(hipStreamSynchronize(s));
    std::vector<unsigned long long> hbuf(tblocks * 64);
    IFD_CHECK_HIP(hipMemcpy(hbuf.data(), tbuf, hbuf.size() * 8, hipMemcpyDeviceToHost));
    IFD_CHECK_HIP(hipFree(tbuf));
    const char* fn = getenv("IFD_TRACE_FILE") ? getenv("IFD_TRACE_FILE") : "conv_trace.bin";
    if (FILE* f = fopen(fn, "wb")) {
      fwrite(hbuf.data(), 8, hbuf.size(), f);
      fclose(f);
    }
    std::string jn = std::string(fn) + ".json";
    if (FILE* f = fopen(jn.c_str(), "w")) {
      fprintf(f, "{\"layer\": \"%s\", \"blocks\": %zu, \"bm\": %d, \"bn\": %d, \"npix_tiles\": %d, "
                 "\"ksplit\": %d, \"nct\": %d, \"chunks\": %d, \"stream\": %d}\n",
              tname, tblocks, p.bm, cw.bn, p.npix_tiles, p.ksplit, cw.cout_pad / cw.bn, cw.cin_pad / 8, (int)use_stream);
      fclose(f);
    }
  }
#endif
  if (!e && p.ksplit > 1) {
    // the reduction writes the output's GroupNorm granule statistics when it has a stat area
    auto it = stat_area_.find(out);
    if (gn_fused_ && epi == EPI_NHWC && it != stat_area_.end() && cw.cout % 4 == 0) {
      p.gstat = it->second;
      int E = 0;
      float cnt = 0.f;
      e = launch_splitk_gstat(p, &E, &cnt, s);
      if (!e) stat_[out] = StatRec{p.gstat, E, cnt, cw.cout};
    } else {
      e = launch_splitk_reduce(p, s);
    }
  }
  if (prof_on_ && e0) prof_end(s, e0, nm, flops, bytes);
  if (e) {
    set_error(std::string("conv launch failed (") + nm + "): " + hipGetErrorString((hipError_t)e));
    return 1;
  }
  return 0;
}

static double gn_bytes(int N, int HW, int C) { return 4.0 * 2.0 * N * (double)HW * C; }

int Model::stats_for(const float* buf, int C, int N, int HW, StatRec* out, hipStream_t s) {
  auto it = stat_.find(buf);
  if (it != stat_.end() && it->second.C == C) {
    *out = it->second;
    return 0;
  }
  auto ar = stat_area_.find(buf);
  IFD_REQUIRE(ar != stat_area_.end(), "GroupNorm input is not a workspace activation buffer");
  StatRec r;
  r.part = ar->second;
  r.C = C;
  int e = launch_gn_granules(buf, C, N, HW, r.part, &r.E, &r.cnt, s);
  if (e) return e;
  stat_[buf] = r;
  *out = r;
  return 0;
}

int Model::run_gn(const float* in0, int c0, const float* in1, int c1, int N, int HW, const GNW& gn, const float* emb,
                  int emb_stride, int emb_off, float* A, float* B, hipStream_t s) {
  if (!gn_fused_ || ((c0 + c1) / 32) % 4 != 0)  // granules are 4 channels: groups must hold whole ones
    return launch_gn(in0, c0, in1, c1, N, HW, wblob_ + gn.g_off, wblob_ + gn.b_off, emb, emb_stride, emb_off,
                     ws_ + ly_.o_part_, A, B, s);
  StatRec r0, r1;
  if (stats_for(in0, c0, N, HW, &r0, s)) return 1;
  if (in1 && stats_for(in1, c1, N, HW, &r1, s)) return 1;
  return launch_gn_finalize2(r0.part, r0.E, r0.cnt, c0, in1 ? r1.part : nullptr, r1.E, r1.cnt, in1 ? c1 : 0, N,
                             wblob_ + gn.g_off, wblob_ + gn.b_off, emb, emb_stride, emb_off, A, B, s);
}

int Model::run_res(const ResP& r, const float* in0, int c0, const float* in1, int c1, int N, int Hin, float* out,
                   hipStream_t s) {
  float* A = ws_ + ly_.o_A_;
  float* Bc = ws_ + ly_.o_B_;
  float* part = ws_ + ly_.o_part_;
  float* t1 = ws_ + ly_.o_t1_;
  const int H = r.xf == XF_UP ? 2 * Hin : (r.xf == XF_DOWN ? Hin / 2 : Hin);
  // ly_.o_pool2_'s pooled residual is valid only within the block whose conv1 wrote it
  pooled_raw_ = nullptr;
  hipEvent_t g0;
  prof_begin(s, &g0, "groupnorm_stats");
  (void)part;
  int e = run_gn(in0, c0, in1, c1, N, Hin * Hin, r.gn1, nullptr, 0, 0, A, Bc, s);
  prof_end(s, g0, "groupnorm_stats", 0.0, gn_bytes(N, Hin * Hin, c0 + c1));
  IFD_LAUNCH_OK(e, "gn");
  if (run_conv(r.conv1, in0, c0, in1, c1, N, Hin, H, r.xf, ACT_AFFINE_SILU, A, Bc, nullptr, 0, nullptr, 0, nullptr, 0,
               0, t1, EPI_NHWC, s))
    return 1;
  prof_begin(s, &g0, "groupnorm_stats");
  e = run_gn(t1, r.cout, nullptr, 0, N, H * H, r.gn2, ws_ + ly_.o_E_, emb_total_, r.emb_off, A, Bc, s);
  prof_end(s, g0, "groupnorm_stats", 0.0, gn_bytes(N, H * H, r.cout));
  IFD_LAUNCH_OK(e, "gn");
  // split modes: skip_connection(x) as its own launch into `out`, then conv2 adds it as its residual
  // in place (each output element's residual is read by the thread that writes it)
  const bool split_mode = prec_ == IFD_PREC_3XF16 || prec_ == IFD_PREC_F16;
  if (split_mode && r.conv2.sk_ok && r.xf == XF_NONE && opt_skip_sep_ > 0 && H >= opt_skip_sep_ &&
      !(opt_x3_off_ & 4)) {
    Skip1x1Params q;
    q.s0 = in0; q.sc0 = c0; q.s1 = in1; q.sc1 = in1 ? c1 : 0;
    q.npix = N * H * H;
    q.cout = r.cout;
    q.wpack = wblob_ + r.conv2.sk_off;
    q.bias = wblob_ + r.conv2.sbias_off;
    q.out = out;
    q.guard = guard_;
    q.ntc = r.conv2.sk_ntc;
    q.nprod = prec_ == IFD_PREC_F16 ? 1 : 3;
    if (skip_x3_eligible(q)) {
      char nm[96] = "";
      const double pix = (double)N * H * H;
      if (prof_on_) {
        if (prof_layers_)
          snprintf(nm, sizeof(nm), "skip_x3 r%d %d+%d->%d", H, c0, q.sc1, r.cout);
        else
          snprintf(nm, sizeof(nm), "skip_x3_kernel<%d,%d>", q.ntc, q.nprod);
      }
      hipEvent_t e0;
      prof_begin(s, &e0, nm);
      const int e2 = launch_skip_x3(q, s);
      if (prof_on_ && e0) prof_end(s, e0, nm, 2.0 * pix * r.cout * (c0 + q.sc1), 4.0 * pix * (c0 + q.sc1 + r.cout));
      if (e2) {
        set_error(std::string("skip launch failed (") + nm + "): " + hipGetErrorString((hipError_t)e2));
        return 1;
      }
      return run_conv(r.conv2_res, t1, r.cout, nullptr, 0, N, H, H, XF_NONE, ACT_AFFINE_SILU, A, Bc, nullptr, 0,
                      nullptr, 0, out, XF_NONE, H, out, EPI_NHWC, s);
    }
  }
  const float* res = r.conv2.has_skip ? nullptr : in0;
  return run_conv(r.conv2, t1, r.cout, nullptr, 0, N, H, H, XF_NONE, ACT_AFFINE_SILU, A, Bc, in0, c0, in1, c1, res,
                  r.xf, Hin, out, EPI_NHWC, s);
}

int Model::run_attn(const AttnP& a, const float* in, int N, int Hin, float* out, hipStream_t s) {
  float* A = ws_ + ly_.o_A_;
  float* Bc = ws_ + ly_.o_B_;
  float* qkv = ws_ + ly_.o_qkv_;
  float* ao = ws_ + ly_.o_ao_;
  const int T = Hin * Hin;
  hipEvent_t g0;
  prof_begin(s, &g0, "groupnorm_stats");
  int e = run_gn(in, a.C, nullptr, 0, N, T, a.gn, nullptr, 0, 0, A, Bc, s);
  prof_end(s, g0, "groupnorm_stats", 0.0, gn_bytes(N, T, a.C));
  IFD_LAUNCH_OK(e, "gn");
  if (run_conv(a.qkv, in, a.C, nullptr, 0, N, Hin, Hin, XF_NONE, ACT_AFFINE, A, Bc, nullptr, 0, nullptr, 0, nullptr, 0,
               0, qkv, EPI_NHWC, s))
    return 1;
  const float scale = (float)(1.0 / std::sqrt(std::sqrt((double)cfg_.num_head_channels)));
  IFD_REQUIRE(cfg_.num_head_channels == 64, "attention kernel is specialised for 64-channel heads");
  prof_begin(s, &g0, "attention_kernel");
  launch_attention(qkv, N, T, a.C, scale, ao, s);
  prof_end(s, g0, "attention_kernel", 4.0 * N * (double)T * T * a.C, 4.0 * N * (double)T * a.C * 4);
  return run_conv(a.proj, ao, a.C, nullptr, 0, N, Hin, Hin, XF_NONE, ACT_NONE, nullptr, nullptr, nullptr, 0, nullptr,
                  0, in, XF_NONE, Hin, out, EPI_NHWC, s);
}

int Model::forward(const float* x, const float* a, const float* m, int pack_mode, const int64_t* t, int B, int H,
                   int W, int epi, float* out6, const StepCoeffs* sc, float* img, const float* gt, const float* mask,
                   const float* noise, const float* known, hipStream_t s) {
  IFD_REQUIRE(H == cfg_.image_size && W == cfg_.image_size, "input size must equal image_size");
  IFD_REQUIRE(B >= 1, "batch must be >= 1");
  if (!finalized_) {
    if (finalize()) return 1;
  }
  if (ensure_workspace(B)) return 1;
  if (!guard_) {
    IFD_CHECK_HIP(hipMalloc(&guard_, 64));
    IFD_CHECK_HIP(hipMemset(guard_, 0, 64));
  }
  const int R = cfg_.image_size;
  const int mc = cfg_.model_channels;
  float* x0 = ws_ + ly_.o_x0_;
  stat_.clear();
  pooled_raw_ = nullptr;
  hipEvent_t p0;
  prof_begin(s, &p0, "input_pack+temb+emb_proj");
  launch_pack_input(x, a, m, pack_mode, B, R * R, x0, s);
  launch_temb(t, wblob_ + freqs_, mc, wblob_ + te_w0_, wblob_ + te_b0_, wblob_ + te_w2_, wblob_ + te_b2_, emb_dim_, B,
              ws_ + ly_.o_h1_, ws_ + ly_.o_emb_, s);
  launch_emb_proj(ws_ + ly_.o_emb_, emb_dim_, B, wblob_ + embw_, wblob_ + embb_, emb_total_, ws_ + ly_.o_E_, s);
  prof_end(s, p0, "input_pack+temb+emb_proj", 2.0 * B * (double)emb_dim_ * (mc + emb_dim_ + emb_total_),
           4.0 * B * (double)R * R * (7 + 16) + 4.0 * emb_dim_ * (double)emb_total_);

  // input blocks
  if (run_conv(conv_in_, x0, 16, nullptr, 0, B, R, R, XF_NONE, ACT_NONE, nullptr, nullptr, nullptr, 0, nullptr, 0,
               nullptr, 0, 0, ws_ + ly_.o_hs_[0], EPI_NHWC, s))
    return 1;
  const float* cur = ws_ + ly_.o_hs_[0];
  int cur_c = in_ch_[0], cur_r = in_res_[0];
  for (size_t i = 1; i < in_blocks_.size(); ++i) {
    const auto& L = in_blocks_[i];
    for (size_t k = 0; k < L.size(); ++k) {
      float* dst = (k + 1 == L.size()) ? ws_ + ly_.o_hs_[i] : ws_ + ly_.o_bufs_[k % 2];
      if (L[k].kind == L_RES) {
        const ResP& r = res_[L[k].idx];
        if (run_res(r, cur, cur_c, nullptr, 0, B, cur_r, dst, s)) return 1;
        cur_c = r.cout;
        if (r.xf == XF_DOWN) cur_r /= 2;
      } else {
        if (run_attn(attn_[L[k].idx], cur, B, cur_r, dst, s)) return 1;
      }
      cur = dst;
    }
  }
  // middle + output blocks: rotate three buffers, never writing the one being read
  int bi = 0;
  auto next_buf = [&](const float* avoid) {
    for (int k = 0; k < 3; ++k) {
      float* b = ws_ + ly_.o_bufs_[(bi + k) % 3];
      if (b != avoid) {
        bi = (bi + k + 1) % 3;
        return b;
      }
    }
    return (float*)nullptr;
  };
  for (auto& L : mid_) {
    float* dst = next_buf(cur);
    if (L.kind == L_RES) {
      if (run_res(res_[L.idx], cur, cur_c, nullptr, 0, B, cur_r, dst, s)) return 1;
    } else {
      if (run_attn(attn_[L.idx], cur, B, cur_r, dst, s)) return 1;
    }
    cur = dst;
  }
  int hs_i = (int)in_blocks_.size() - 1;
  for (auto& blk : out_blocks_) {
    for (size_t k = 0; k < blk.size(); ++k) {
      const LayerP& L = blk[k];
      float* dst = next_buf(cur);
      if (L.kind == L_RES) {
        const ResP& r = res_[L.idx];
        if (k == 0) {
          const float* skip = ws_ + ly_.o_hs_[hs_i];
          if (run_res(r, cur, cur_c, skip, in_ch_[hs_i], B, cur_r, dst, s)) return 1;
          --hs_i;
        } else {
          if (run_res(r, cur, cur_c, nullptr, 0, B, cur_r, dst, s)) return 1;
        }
        cur_c = r.cout;
        if (r.xf == XF_UP) cur_r *= 2;
      } else {
        if (run_attn(attn_[L.idx], cur, B, cur_r, dst, s)) return 1;
      }
      cur = dst;
    }
  }
  // out: GN -> SiLU -> conv 3x3 -> [B,6,H,W] (or the fused sampler update)
  float* A = ws_ + ly_.o_A_;
  float* Bc = ws_ + ly_.o_B_;
  prof_begin(s, &p0, "groupnorm_stats");
  int e = run_gn(cur, cur_c, nullptr, 0, B, R * R, gn_out_, nullptr, 0, 0, A, Bc, s);
  prof_end(s, p0, "groupnorm_stats", 0.0, gn_bytes(B, R * R, cur_c));
  IFD_LAUNCH_OK(e, "gn");
  return run_conv(conv_out_, cur, cur_c, nullptr, 0, B, R, R, XF_NONE, ACT_AFFINE_SILU, A, Bc, nullptr, 0, nullptr, 0,
                  nullptr, 0, 0, out6, epi, s, sc, img, gt, mask, noise, known);
}

}  // namespace ifd
