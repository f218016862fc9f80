// Native image augmentation + normalisation for ImageRecordIter (see image_aug.cc).
#pragma once
#include <cstdint>
#include <random>
#include <string>
#include <vector>

namespace mxamd {

// Interleaved 8-bit image (HWC, RGB / gray / RGBA).
struct Image {
  int h = 0, w = 0, c = 0;
  std::vector<uint8_t> px;
  Image() = default;
  Image(int h_, int w_, int c_, uint8_t fill = 0) : h(h_), w(w_), c(c_), px(size_t(h_) * w_ * c_, fill) {}
  uint8_t* row(int y) { return px.data() + size_t(y) * w * c; }
  const uint8_t* row(int y) const { return px.data() + size_t(y) * w * c; }
};

// Augmentation parameters: the reference's DefaultImageAugmentParam plus the
// normalisation parameters of ImageNormalizeParam (image_iter_common.h).
struct AugParam {
  int out_c = 3, out_h = 0, out_w = 0;      // data_shape
  int resize = -1;
  bool rand_crop = false;
  bool random_resized_crop = false;
  int max_rotate_angle = 0;
  float max_aspect_ratio = 0.f;
  bool has_min_aspect_ratio = false;
  float min_aspect_ratio = 0.f;
  float max_shear_ratio = 0.f;
  int max_crop_size = -1, min_crop_size = -1;
  float max_random_scale = 1.f, min_random_scale = 1.f;
  float max_random_area = 1.f, min_random_area = 1.f;
  float min_img_size = 0.f, max_img_size = 1e10f;
  float brightness = 0.f, contrast = 0.f, saturation = 0.f;
  float pca_noise = 0.f;
  int random_h = 0, random_s = 0, random_l = 0;
  int rotate = -1;
  std::vector<int> rotate_list;
  int fill_value = 255;
  int inter_method = 1;
  int pad = 0;
  // normalisation (applied while writing the output tensor)
  bool mirror = false, rand_mirror = false;
  float mean[4] = {0.f, 0.f, 0.f, 0.f};
  float std_[4] = {1.f, 1.f, 1.f, 1.f};
  float scale = 1.f;
  float max_random_contrast = 0.f, max_random_illumination = 0.f;
  std::vector<float> mean_img;                // optional (out_c, out_h, out_w) mean image
};

// Output element type / layout of the batch slot.
enum class OutType { kFloat32 = 0, kUint8 = 1, kInt8 = 2 };

// Validates parameter combinations the reference CHECK-fails on; returns "" or a message.
std::string CheckAugParam(const AugParam& p);

// Geometric + colour augmentation of one decoded image (output is out_h x out_w).
Image Augment(const Image& src, const AugParam& p, std::mt19937& rng);

// Mirror + mean/std/scale (+random contrast/illumination) while writing into a
// batch slot laid out CHW (nchw=true) or HWC.
void WriteNormalized(const Image& img, const AugParam& p, std::mt19937& rng, void* out, OutType t,
                     bool nchw);

// Plain resize (used by the mean-image pass and image.imresize).
Image Resize(const Image& src, int w, int h, int inter);

}  // namespace mxamd
