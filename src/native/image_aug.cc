// Native image augmentation for ImageRecordIter.
//
// Parity: src/io/image_aug_default.cc (DefaultImageAugmenter::Process: resize,
// affine rotate/shear/scale/aspect, pad, random-resized-crop, random crop size,
// centre/random crop, brightness/contrast/saturation jitter, HSL jitter, PCA
// lighting noise, interpolation methods 0-4/9/10) and
// src/io/iter_image_recordio_2.cc:376 (ProcessImage: mirror, mean/std/scale,
// random contrast/illumination, int8/uint8 outputs).
//
// The reference runs these through OpenCV on BGR mats; this is a self-contained
// implementation on interleaved RGB bytes (PIL decodes RGB) with separable
// resamplers and an inverse-mapped affine warp.  It runs on the data-loader
// engine's worker threads without the GIL, writing straight into the batch
// slot (pinned host memory when the iterator feeds a GPU), so the only copy of
// a decoded image is the one into the batch.  Deliberate differences: grey for
// the contrast/saturation jitter uses RGB luma weights on RGB data (the
// reference applies RGB weights to BGR data), and cubic/Lanczos warps sample
// bilinearly (resizes honour all five methods).
#include "image_aug.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <stdexcept>

namespace mxamd {

namespace {

constexpr int kNN = 0, kLinear = 1, kCubic = 2, kArea = 3, kLanczos = 4;

inline uint8_t Sat8(float v) {
  int i = static_cast<int>(std::lrintf(v));
  return static_cast<uint8_t>(std::min(255, std::max(0, i)));
}

inline int8_t SatS8(int v) { return static_cast<int8_t>(std::min(127, std::max(-128, v))); }

// 9 = auto (cubic to enlarge, area to shrink, linear otherwise), 10 = random.
int ResolveInter(int m, int ow, int oh, int nw, int nh, std::mt19937& rng) {
  if (m == 9) {
    if (nw > ow && nh > oh) return kCubic;
    if (nw < ow && nh < oh) return kArea;
    return kLinear;
  }
  if (m == 10) return std::uniform_int_distribution<int>(0, 4)(rng);
  return m;
}

float CubicW(float x) {
  const float A = -0.75f;
  x = std::fabs(x);
  if (x < 1.f) return ((A + 2.f) * x - (A + 3.f)) * x * x + 1.f;
  if (x < 2.f) return ((A * x - 5.f * A) * x + 8.f * A) * x - 4.f * A;
  return 0.f;
}

float LanczosW(float x) {
  if (std::fabs(x) < 1e-6f) return 1.f;
  if (std::fabs(x) >= 4.f) return 0.f;
  const float px = static_cast<float>(M_PI) * x;
  return 4.f * std::sin(px) * std::sin(px / 4.f) / (px * px);
}

// Per output coordinate: n (source index, weight) taps.
struct Taps {
  int n = 1;
  std::vector<int> idx;
  std::vector<float> w;
};

Taps MakeTaps(int in, int out, int inter) {
  Taps t;
  const double sc = static_cast<double>(in) / out;
  if (inter == kArea && sc > 1.0) {
    t.n = static_cast<int>(std::ceil(sc)) + 1;
    t.idx.assign(size_t(out) * t.n, 0);
    t.w.assign(size_t(out) * t.n, 0.f);
    for (int o = 0; o < out; ++o) {
      const double a = o * sc, b = (o + 1) * sc;
      int k = 0;
      for (int i = static_cast<int>(std::floor(a)); i < std::ceil(b) && k < t.n; ++i) {
        const double lo = std::max(a, double(i)), hi = std::min(b, double(i) + 1.0);
        if (hi <= lo) continue;
        t.idx[size_t(o) * t.n + k] = std::min(i, in - 1);
        t.w[size_t(o) * t.n + k] = static_cast<float>((hi - lo) / sc);
        ++k;
      }
    }
    return t;
  }
  if (inter == kNN) {
    t.idx.resize(out);
    t.w.assign(out, 1.f);
    for (int o = 0; o < out; ++o) t.idx[o] = std::min(static_cast<int>(std::floor(o * sc)), in - 1);
    return t;
  }
  t.n = inter == kCubic ? 4 : inter == kLanczos ? 8 : 2;   // area-enlarge samples linearly
  t.idx.resize(size_t(out) * t.n);
  t.w.resize(size_t(out) * t.n);
  for (int o = 0; o < out; ++o) {
    const double ctr = (o + 0.5) * sc - 0.5;
    const int first = static_cast<int>(std::floor(ctr)) - (t.n / 2 - 1);
    float sum = 0.f;
    for (int k = 0; k < t.n; ++k) {
      const int i = first + k;
      const float d = static_cast<float>(i - ctr);
      float w = t.n == 2 ? std::max(0.f, 1.f - std::fabs(d)) : t.n == 4 ? CubicW(d) : LanczosW(d);
      t.idx[size_t(o) * t.n + k] = std::min(std::max(i, 0), in - 1);
      t.w[size_t(o) * t.n + k] = w;
      sum += w;
    }
    if (sum != 0.f)
      for (int k = 0; k < t.n; ++k) t.w[size_t(o) * t.n + k] /= sum;
  }
  return t;
}

Image Crop(const Image& s, int x, int y, int w, int h) {
  Image d(h, w, s.c);
  for (int r = 0; r < h; ++r)
    std::copy_n(s.row(y + r) + size_t(x) * s.c, size_t(w) * s.c, d.row(r));
  return d;
}

// dst(x, y) = src(M^-1 (x, y)), constant border.
Image WarpAffine(const Image& s, const float M[6], int W, int H, int inter, int fill) {
  const float det = M[0] * M[4] - M[1] * M[3];
  if (std::fabs(det) < 1e-12f) throw std::runtime_error("degenerate affine transform");
  const float ia = M[4] / det, ib = -M[1] / det, ic = -M[3] / det, id = M[0] / det;
  const float itx = -(ia * M[2] + ib * M[5]), ity = -(ic * M[2] + id * M[5]);
  Image d(H, W, s.c);
  const uint8_t fv = static_cast<uint8_t>(std::min(255, std::max(0, fill)));
  const int C = s.c;
  for (int y = 0; y < H; ++y) {
    uint8_t* out = d.row(y);
    for (int x = 0; x < W; ++x, out += C) {
      const float sx = ia * x + ib * y + itx, sy = ic * x + id * y + ity;
      if (inter == kNN) {
        const int ix = static_cast<int>(std::lrintf(sx)), iy = static_cast<int>(std::lrintf(sy));
        if (ix < 0 || iy < 0 || ix >= s.w || iy >= s.h) {
          std::fill_n(out, C, fv);
        } else {
          std::copy_n(s.row(iy) + size_t(ix) * C, C, out);
        }
        continue;
      }
      const int x0 = static_cast<int>(std::floor(sx)), y0 = static_cast<int>(std::floor(sy));
      const float fx = sx - x0, fy = sy - y0;
      if (x0 < -1 || y0 < -1 || x0 >= s.w || y0 >= s.h) {
        std::fill_n(out, C, fv);
        continue;
      }
      const float wts[4] = {(1 - fx) * (1 - fy), fx * (1 - fy), (1 - fx) * fy, fx * fy};
      const int xs[4] = {x0, x0 + 1, x0, x0 + 1}, ys[4] = {y0, y0, y0 + 1, y0 + 1};
      for (int ch = 0; ch < C; ++ch) {
        float acc = 0.f;
        for (int k = 0; k < 4; ++k) {
          const bool in = xs[k] >= 0 && ys[k] >= 0 && xs[k] < s.w && ys[k] < s.h;
          acc += wts[k] * (in ? s.row(ys[k])[size_t(xs[k]) * C + ch] : fv);
        }
        out[ch] = Sat8(acc);
      }
    }
  }
  return d;
}

inline float Luma(const uint8_t* p) { return 0.299f * p[0] + 0.587f * p[1] + 0.114f * p[2]; }

void RgbToHls(const uint8_t* p, int* hls) {
  const float r = p[0] / 255.f, g = p[1] / 255.f, b = p[2] / 255.f;
  const float vmax = std::max(r, std::max(g, b)), vmin = std::min(r, std::min(g, b));
  float diff = vmax - vmin, h = 0.f, s = 0.f;
  const float l = (vmax + vmin) * 0.5f;
  if (diff > FLT_EPSILON) {
    s = l < 0.5f ? diff / (vmax + vmin) : diff / (2.f - vmax - vmin);
    diff = 60.f / diff;
    if (vmax == r)
      h = (g - b) * diff;
    else if (vmax == g)
      h = (b - r) * diff + 120.f;
    else
      h = (r - g) * diff + 240.f;
    if (h < 0.f) h += 360.f;
  }
  hls[0] = Sat8(h * 0.5f);
  hls[1] = Sat8(l * 255.f);
  hls[2] = Sat8(s * 255.f);
}

void HlsToRgb(const int* hls, uint8_t* p) {
  float h = hls[0] * 2.f;
  const float l = hls[1] / 255.f, s = hls[2] / 255.f;
  float r = l, g = l, b = l;
  if (s != 0.f) {
    static const int kSector[6][3] = {{1, 3, 0}, {1, 0, 2}, {3, 0, 1}, {0, 2, 1}, {0, 1, 3}, {2, 1, 0}};
    const float p2 = l <= 0.5f ? l * (1.f + s) : l + s - l * s;
    const float p1 = 2.f * l - p2;
    h /= 60.f;
    while (h < 0.f) h += 6.f;
    while (h >= 6.f) h -= 6.f;
    const int sec = static_cast<int>(h);
    h -= sec;
    const float tab[4] = {p2, p1, p1 + (p2 - p1) * (1.f - h), p1 + (p2 - p1) * h};
    b = tab[kSector[sec][0]];
    g = tab[kSector[sec][1]];
    r = tab[kSector[sec][2]];
  }
  p[0] = Sat8(r * 255.f);
  p[1] = Sat8(g * 255.f);
  p[2] = Sat8(b * 255.f);
}

void ColorJitter(Image& im, const AugParam& p, std::mt19937& rng) {
  const float ab = 1.f + std::uniform_real_distribution<float>(-p.brightness, p.brightness)(rng);
  const float ac = 1.f + std::uniform_real_distribution<float>(-p.contrast, p.contrast)(rng);
  const float as = 1.f + std::uniform_real_distribution<float>(-p.saturation, p.saturation)(rng);
  int order[3] = {0, 1, 2};
  std::shuffle(order, order + 3, rng);
  const size_t n = size_t(im.h) * im.w;
  for (int op : order) {
    uint8_t* px = im.px.data();
    if (op == 0) {
      for (size_t i = 0; i < n * 3; ++i) px[i] = Sat8(px[i] * ab);
    } else if (op == 1) {
      double mean = 0.0;
      for (size_t i = 0; i < n; ++i) mean += Sat8(Luma(px + 3 * i));
      const float m = static_cast<float>(mean / std::max<size_t>(n, 1));
      for (size_t i = 0; i < n * 3; ++i) px[i] = Sat8(px[i] * ac + (1.f - ac) * m);
    } else {
      for (size_t i = 0; i < n; ++i) {
        const float gr = Sat8(Luma(px + 3 * i));
        for (int k = 0; k < 3; ++k) px[3 * i + k] = Sat8(px[3 * i + k] * as + gr * (1.f - as));
      }
    }
  }
}

void HslJitter(Image& im, const AugParam& p, std::mt19937& rng) {
  std::uniform_real_distribution<float> u(0.f, 1.f);
  // the reference's approximate Gaussian: (u + 4u') / 5
  float rh = u(rng); rh += 4 * u(rng); rh /= 5;
  float rs = u(rng); rs += 4 * u(rng); rs /= 5;
  float rl = u(rng); rl += 4 * u(rng); rl /= 5;
  const int dh = static_cast<int>(rh * p.random_h * 2 - p.random_h);
  const int ds = static_cast<int>(rs * p.random_s * 2 - p.random_s);
  const int dl = static_cast<int>(rl * p.random_l * 2 - p.random_l);
  const int delta[3] = {dh, dl, ds}, limit[3] = {180, 255, 255};
  const size_t n = size_t(im.h) * im.w;
  uint8_t* px = im.px.data();
  for (size_t i = 0; i < n; ++i) {
    int hls[3];
    RgbToHls(px + 3 * i, hls);
    for (int k = 0; k < 3; ++k) hls[k] = std::max(0, std::min(limit[k], hls[k] + delta[k]));
    HlsToRgb(hls, px + 3 * i);
  }
}

void PcaNoise(Image& im, const AugParam& p, std::mt19937& rng) {
  // eigenvalue-scaled eigenvectors of ImageNet RGB covariance (rows R, G, B)
  static const float kEig[3][3] = {{55.46f * -0.5675f, 4.794f * 0.7192f, 1.148f * 0.4009f},
                                   {55.46f * -0.5808f, 4.794f * -0.0045f, 1.148f * -0.8140f},
                                   {55.46f * -0.5836f, 4.794f * -0.6948f, 1.148f * 0.4203f}};
  std::normal_distribution<float> nd(0.f, p.pca_noise);
  const float a0 = nd(rng), a1 = nd(rng), a2 = nd(rng);
  float add[3];
  for (int k = 0; k < 3; ++k) add[k] = kEig[k][0] * a0 + kEig[k][1] * a1 + kEig[k][2] * a2;
  const size_t n = size_t(im.h) * im.w;
  uint8_t* px = im.px.data();
  for (size_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) {
      const int v = static_cast<int>(px[3 * i + k] + add[k]);
      px[3 * i + k] = static_cast<uint8_t>(std::max(0, std::min(255, v)));
    }
}

bool ValidResizeInter(int m) { return (m >= 0 && m <= 4) || m == 9 || m == 10; }
bool ValidWarpInter(int m) { return (m >= 1 && m <= 4) || m == 9 || m == 10; }

Image ConvertChannels(const Image& s, int c) {
  if (s.c == c) return s;
  Image d(s.h, s.w, c);
  const size_t n = size_t(s.h) * s.w;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t* a = s.px.data() + i * s.c;
    uint8_t* b = d.px.data() + i * c;
    uint8_t rgb[3];
    if (s.c == 1) {
      rgb[0] = rgb[1] = rgb[2] = a[0];
    } else {
      rgb[0] = a[0]; rgb[1] = a[1]; rgb[2] = a[2];
    }
    if (c == 1) {
      b[0] = s.c == 1 ? a[0] : Sat8(Luma(rgb));
    } else {
      b[0] = rgb[0]; b[1] = rgb[1]; b[2] = rgb[2];
      if (c == 4) b[3] = s.c == 4 ? a[3] : 255;
    }
  }
  return d;
}

}  // namespace

Image Resize(const Image& s, int W, int H, int inter) {
  if (W <= 0 || H <= 0) throw std::runtime_error("resize to an empty image");
  if (W == s.w && H == s.h) return s;
  const Taps tx = MakeTaps(s.w, W, inter), ty = MakeTaps(s.h, H, inter);
  const int C = s.c;
  std::vector<float> tmp(size_t(s.h) * W * C);
  for (int y = 0; y < s.h; ++y) {
    const uint8_t* in = s.row(y);
    float* o = tmp.data() + size_t(y) * W * C;
    for (int x = 0; x < W; ++x)
      for (int ch = 0; ch < C; ++ch) {
        float acc = 0.f;
        for (int k = 0; k < tx.n; ++k) acc += tx.w[size_t(x) * tx.n + k] * in[size_t(tx.idx[size_t(x) * tx.n + k]) * C + ch];
        o[size_t(x) * C + ch] = acc;
      }
  }
  Image d(H, W, C);
  for (int y = 0; y < H; ++y) {
    uint8_t* o = d.row(y);
    for (size_t j = 0; j < size_t(W) * C; ++j) {
      float acc = 0.f;
      for (int k = 0; k < ty.n; ++k) acc += ty.w[size_t(y) * ty.n + k] * tmp[size_t(ty.idx[size_t(y) * ty.n + k]) * W * C + j];
      o[j] = Sat8(acc);
    }
  }
  return d;
}

std::string CheckAugParam(const AugParam& p) {
  if (p.out_c != 1 && p.out_c != 3 && p.out_c != 4)
    return "ImageRecordIter: data_shape[0] must be 1, 3 or 4 channels, got " + std::to_string(p.out_c);
  if (p.out_h <= 0 || p.out_w <= 0) return "ImageRecordIter: data_shape must be positive";
  if (!ValidResizeInter(p.inter_method)) return "invalid inter_method: valid value 0,1,2,3,9,10";
  if (p.random_resized_crop &&
      (p.min_random_scale != 1.f || p.max_random_scale != 1.f || p.min_crop_size != -1 ||
       p.max_crop_size != -1 || p.rand_crop))
    return "Setting random_resized_crop to true conflicts with min_random_scale, max_random_scale, "
           "min_crop_size, max_crop_size, and rand_crop.";
  if (p.max_crop_size < p.min_crop_size) return "max_crop_size must be >= min_crop_size";
  return "";
}

Image Augment(const Image& src0, const AugParam& p, std::mt19937& rng) {
  const std::string err = CheckAugParam(p);
  if (!err.empty()) throw std::runtime_error(err);
  Image src = ConvertChannels(src0, p.out_c);
  float max_ar, min_ar;
  if (p.has_min_aspect_ratio) {
    max_ar = p.max_aspect_ratio;
    min_ar = p.min_aspect_ratio;
  } else {
    max_ar = 1.f + p.max_aspect_ratio;
    min_ar = 1.f - p.max_aspect_ratio;
  }
  Image res;
  if (p.resize != -1) {
    int nh, nw;
    if (src.h > src.w) {
      nh = p.resize * src.h / src.w;
      nw = p.resize;
    } else {
      nh = p.resize;
      nw = p.resize * src.w / src.h;
    }
    res = Resize(src, nw, nh, ResolveInter(p.inter_method, src.w, src.h, nw, nh, rng));
  } else {
    res = std::move(src);
  }

  // rotation / shear / scale / aspect as one affine warp
  if (p.max_rotate_angle > 0 || p.max_shear_ratio > 0.f || p.rotate > 0 || !p.rotate_list.empty() ||
      p.max_random_scale != 1.f || p.min_random_scale != 1.f ||
      (!p.random_resized_crop && (min_ar != 1.f || max_ar != 1.f)) || p.max_img_size != 1e10f ||
      p.min_img_size != 0.f) {
    if (!ValidWarpInter(p.inter_method)) throw std::runtime_error("invalid inter_method: valid value 0,1,2,3,9,10");
    std::uniform_real_distribution<float> u(0.f, 1.f);
    const float shear = u(rng) * p.max_shear_ratio * 2 - p.max_shear_ratio;
    int angle = std::uniform_int_distribution<int>(-p.max_rotate_angle, p.max_rotate_angle)(rng);
    if (p.rotate > 0) angle = p.rotate;
    if (!p.rotate_list.empty())
      angle = p.rotate_list[std::uniform_int_distribution<int>(0, int(p.rotate_list.size()) - 1)(rng)];
    const float ca = std::cos(angle / 180.0 * M_PI), sa = std::sin(angle / 180.0 * M_PI);
    float scale = 1.f, ratio = 1.f;
    if (!p.random_resized_crop) {
      scale = u(rng) * (p.max_random_scale - p.min_random_scale) + p.min_random_scale;
      ratio = u(rng) * (max_ar - min_ar) + min_ar;
    }
    const float hs = 2 * scale / (1 + ratio), ws = ratio * hs;
    const float nw = std::max(p.min_img_size, std::min(p.max_img_size, scale * res.w));
    const float nh = std::max(p.min_img_size, std::min(p.max_img_size, scale * res.h));
    float M[6];
    M[0] = hs * ca - shear * sa * ws;
    M[3] = -sa * ws;
    M[1] = hs * sa + shear * ca * ws;
    M[4] = ca * ws;
    M[2] = (nw - (M[0] * res.w + M[1] * res.h)) / 2;
    M[5] = (nh - (M[3] * res.w + M[4] * res.h)) / 2;
    const int inter = ResolveInter(p.inter_method, res.w, res.h, int(nw), int(nh), rng);
    res = WarpAffine(res, M, std::max(1, int(nw)), std::max(1, int(nh)), inter, p.fill_value);
  }

  if (p.pad > 0) {
    Image padded(res.h + 2 * p.pad, res.w + 2 * p.pad, res.c,
                 static_cast<uint8_t>(std::min(255, std::max(0, p.fill_value))));
    for (int y = 0; y < res.h; ++y)
      std::copy_n(res.row(y), size_t(res.w) * res.c, padded.row(y + p.pad) + size_t(p.pad) * res.c);
    res = std::move(padded);
  }

  bool cropped = false;
  if (p.random_resized_crop) {
    if (p.max_random_area != 1.f || p.min_random_area != 1.f || max_ar != 1.f || min_ar != 1.f) {
      if (!(min_ar > 0.f) || p.min_random_area > p.max_random_area || min_ar > max_ar)
        throw std::runtime_error("random_resized_crop: invalid area / aspect-ratio range");
      std::uniform_real_distribution<float> ua(p.min_random_area, p.max_random_area);
      std::uniform_real_distribution<float> ur(min_ar, max_ar);
      std::uniform_real_distribution<float> u(0.f, 1.f);
      const float area = float(res.h) * res.w;
      for (int i = 0; i < 10; ++i) {
        const float target = area * ua(rng);
        const float r = ur(rng);
        int yh = static_cast<int>(std::round(std::sqrt(target / r)));
        int xw = static_cast<int>(std::round(std::sqrt(target * r)));
        if (u(rng) > 0.5f) std::swap(yh, xw);
        if (yh <= res.h && xw <= res.w && yh > 0 && xw > 0) {
          const int y0 = std::uniform_int_distribution<int>(0, res.h - yh)(rng);
          const int x0 = std::uniform_int_distribution<int>(0, res.w - xw)(rng);
          const int inter = ResolveInter(p.inter_method, xw, yh, p.out_w, p.out_h, rng);
          res = Resize(Crop(res, x0, y0, xw, yh), p.out_w, p.out_h, inter);
          cropped = true;
          break;
        }
      }
    }
  } else if (p.max_crop_size != -1 || p.min_crop_size != -1) {
    if (res.w < p.max_crop_size || res.h < p.max_crop_size)
      throw std::runtime_error("input image size smaller than max_crop_size");
    const int cs = std::uniform_int_distribution<int>(p.min_crop_size, p.max_crop_size)(rng);
    int y = res.h - cs, x = res.w - cs;
    if (p.rand_crop) {
      y = std::uniform_int_distribution<int>(0, y)(rng);
      x = std::uniform_int_distribution<int>(0, x)(rng);
    } else {
      y /= 2;
      x /= 2;
    }
    const int inter = ResolveInter(p.inter_method, cs, cs, p.out_w, p.out_h, rng);
    res = Resize(Crop(res, x, y, cs, cs), p.out_w, p.out_h, inter);
    cropped = true;
  }

  if (!cropped) {
    const int inter = ResolveInter(p.inter_method, res.w, res.h, p.out_w, p.out_h, rng);
    if (res.h < p.out_h) {
      const int nc = static_cast<int>(float(p.out_h) / res.h * res.w);
      res = Resize(res, std::max(1, nc), p.out_h, inter);
    }
    if (res.w < p.out_w) {
      const int nr = static_cast<int>(float(p.out_w) / res.w * res.h);
      res = Resize(res, p.out_w, std::max(1, nr), inter);
    }
    if (res.h < p.out_h || res.w < p.out_w) throw std::runtime_error("input image size smaller than input shape");
    int y = res.h - p.out_h, x = res.w - p.out_w;
    if (p.rand_crop) {
      y = std::uniform_int_distribution<int>(0, y)(rng);
      x = std::uniform_int_distribution<int>(0, x)(rng);
    } else {
      y /= 2;
      x /= 2;
    }
    if (x != 0 || y != 0 || res.w != p.out_w || res.h != p.out_h) res = Crop(res, x, y, p.out_w, p.out_h);
  }

  if (res.c == 3) {
    if (p.brightness > 0.f || p.contrast > 0.f || p.saturation > 0.f) ColorJitter(res, p, rng);
    if (p.random_h != 0 || p.random_s != 0 || p.random_l != 0) HslJitter(res, p, rng);
    if (p.pca_noise > 0.f) PcaNoise(res, p, rng);
  }
  return res;
}

void WriteNormalized(const Image& img, const AugParam& p, std::mt19937& rng, void* out, OutType t,
                     bool nchw) {
  if (img.h != p.out_h || img.w != p.out_w || img.c != p.out_c)
    throw std::runtime_error("augmented image does not match data_shape");
  const bool mirrored = (p.rand_mirror && std::bernoulli_distribution(0.5)(rng)) || p.mirror;
  float contrast = 1.f, illum = 0.f;
  if (t != OutType::kUint8) {
    std::uniform_real_distribution<float> u(0.f, 1.f);
    contrast = (u(rng) * p.max_random_contrast * 2 - p.max_random_contrast + 1) * p.scale;
    illum = (u(rng) * p.max_random_illumination * 2 - p.max_random_illumination) * p.scale;
  }
  const int C = img.c, H = img.h, W = img.w;
  float mult[4], bias[4];
  int mean_i[4];
  for (int k = 0; k < C; ++k) {
    mult[k] = contrast / p.std_[k];
    bias[k] = illum / p.std_[k];
    mean_i[k] = static_cast<int>(std::round(p.mean[k]));
  }
  const bool has_mean_img = p.mean_img.size() == size_t(C) * H * W;
  for (int i = 0; i < H; ++i) {
    const uint8_t* row = img.row(i);
    for (int j = 0; j < W; ++j) {
      const int jj = mirrored ? W - 1 - j : j;
      for (int k = 0; k < C; ++k) {
        const size_t o = nchw ? (size_t(k) * H + i) * W + jj : (size_t(i) * W + jj) * C + k;
        const uint8_t v = row[size_t(j) * C + k];
        const float m = has_mean_img ? p.mean_img[(size_t(k) * H + i) * W + j] : p.mean[k];
        switch (t) {
          case OutType::kFloat32:
            static_cast<float*>(out)[o] = (v - m) * mult[k] + bias[k];
            break;
          case OutType::kUint8:
            static_cast<uint8_t*>(out)[o] = v;
            break;
          case OutType::kInt8:
            static_cast<int8_t*>(out)[o] =
                SatS8(v - (has_mean_img ? static_cast<int>(std::round(m)) : mean_i[k]));
            break;
        }
      }
    }
  }
}

}  // namespace mxamd
