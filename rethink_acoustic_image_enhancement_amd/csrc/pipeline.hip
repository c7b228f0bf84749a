// Pre/post-processing around the forward, on the GPU instead of host numpy.
//
// preprocess (KDLAE/KDLAE_T.ipynb, load_image_as_tensor + the padding cell; ASDQE ToTensor):
//   u8 HWC (1, 3 or 4 channels; cv2 BGR optional) -> f32 NCHW / 255, alpha dropped, reflect-padded on
//   the bottom/right to (H, W), plus the constant denoise_rate map [B,1,H,W].
// frames (KDLAE/KDLAE-S.ipynb load_consecutive_stack + its padding cell): F frames of u8 HWC (gray,
//   or BGR/BGRA as cv2.imread returns them) -> cv2 COLOR_BGR2GRAY -> f32 [B,F,H,W] / 255, reflect-
//   padded to a multiple of 32; the output cell is the same postprocess with C = F frames.
// postprocess (the clamp / crop / img_as_ubyte / zero-mask cell):
//   clamp(x, 0, 1) -> crop to (h*s, w*s) -> rint(x * 255) as u8 HWC; pixels whose input pixel
//   (nearest, for the x2 SR output) is black in every channel are set to 0.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "runtime.h"

namespace kdlae {

namespace {

// torch.nn.functional.pad(mode='reflect') index map for a pad that is shorter than the input
__device__ __forceinline__ int reflect_idx(int i, int n) { return i < n ? i : 2 * (n - 1) - i; }

// cv2.cvtColor(COLOR_BGR2GRAY) on 8-bit data: fixed point, Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14
// (OpenCV's yuv_shift = 14 and its B2Y / G2Y / R2Y coefficients; alpha ignored)
__device__ __forceinline__ uint8_t bgr2gray_u8(const uint8_t* px) {
  return (uint8_t)((1868u * px[0] + 9617u * px[1] + 4899u * px[2] + 8192u) >> 14);
}

__global__ __launch_bounds__(256) void preprocess_u8_kernel(PreParams p) {
  const long long total = (long long)p.B * p.H * p.W;
  const long long HW = (long long)p.H * p.W;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int b = (int)(idx / HW);
    const int rem = (int)(idx - (long long)b * HW);
    const int y = rem / p.W, x = rem - (rem / p.W) * p.W;
    const int sy = reflect_idx(y, p.h), sx = reflect_idx(x, p.w);
    const uint8_t* px = p.in + (((long long)b * p.h + sy) * p.w + sx) * p.cin;
    if (p.gray) {
      p.img[(long long)b * HW + rem] = (float)(p.cin >= 3 ? bgr2gray_u8(px) : px[0]) / 255.0f;
      continue;
    }
    for (int c = 0; c < p.cout; ++c) {
      const int sc = (p.bgr && p.cin >= 3 && c < 3) ? 2 - c : c;
      p.img[((long long)b * p.cout + c) * HW + rem] = (float)px[sc] / 255.0f;
    }
    if (p.rate_map) p.rate_map[idx] = p.rate[b];
  }
}

__global__ __launch_bounds__(256) void postprocess_u8_kernel(PostParams p) {
  const int ho = p.h * p.scale, wo = p.w * p.scale;
  const long long total = (long long)p.B * ho * wo;
  const long long HWs = (long long)p.Hs * p.Ws;
  for (long long idx = blockIdx.x * 256LL + threadIdx.x; idx < total; idx += (long long)gridDim.x * 256) {
    const int b = (int)(idx / ((long long)ho * wo));
    const int rem = (int)(idx - (long long)b * ho * wo);
    const int y = rem / wo, x = rem - (rem / wo) * wo;
    bool black = false;
    if (p.lq) {
      const uint8_t* q = p.lq + (((long long)b * p.h + y / p.scale) * p.w + x / p.scale) * p.cin;
      black = true;
      for (int c = 0; c < (p.cin == 4 ? 3 : p.cin); ++c) black = black && q[c] == 0;
    }
    uint8_t* o = p.out + idx * p.C;
    for (int c = 0; c < p.C; ++c) {
      float v = p.src[((long long)b * p.C + c) * HWs + (long long)y * p.Ws + x];
      v = fminf(fmaxf(v, 0.0f), 1.0f);
      o[c] = black ? (uint8_t)0 : (uint8_t)rintf(v * 255.0f);
    }
  }
}

long long grid_for(long long total) {
  long long blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  return blocks < 1 ? 1 : blocks;
}

}  // namespace

hipError_t launch_preprocess_u8(const PreParams& p, hipStream_t s) {
  if (p.h > p.H || p.w > p.W || p.H - p.h >= p.h || p.W - p.w >= p.w || p.cout < 1 || p.cout > p.cin ||
      p.cin > 4 || (p.gray && p.cout != 1))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(preprocess_u8_kernel, dim3((unsigned)grid_for((long long)p.B * p.H * p.W)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_postprocess_u8(const PostParams& p, hipStream_t s) {
  if (p.h * p.scale > p.Hs || p.w * p.scale > p.Ws || p.C < 1 || p.C > 64 || (p.scale != 1 && p.scale != 2))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(postprocess_u8_kernel, dim3((unsigned)grid_for((long long)p.B * p.h * p.scale * p.w * p.scale)),
                     dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace kdlae

extern "C" {

int kdlae_preprocess_u8(const uint8_t* images, int B, int h, int w, int channels, int bgr, int multiple,
                        const float* rate, float* img, float* rate_map, void* stream) {
  using namespace kdlae;
  if (!images || !img || B <= 0 || h <= 0 || w <= 0 || multiple <= 0) return fail(KDLAE_ESTATE, "bad argument");
  if (channels != 1 && channels != 3 && channels != 4) return fail(KDLAE_EINVAL_SHAPE, "channels must be 1, 3 or 4");
  if (rate_map && !rate) return fail(KDLAE_ESTATE, "rate_map needs rate");
  int H, W;
  kdlae_padded_size(h, w, multiple, &H, &W);
  if (H - h >= h || W - w >= w) return fail(KDLAE_EINVAL_SHAPE, "image smaller than its reflect padding");
  PreParams p{images, B, h, w, channels, channels == 4 ? 3 : channels, bgr, 0, H, W, img, rate, rate_map};
  HIPCHK(launch_preprocess_u8(p, reinterpret_cast<hipStream_t>(stream)));
  return KDLAE_OK;
}

int kdlae_frames_preprocess_u8(const uint8_t* frames, int B, int F, int h, int w, int channels, int multiple,
                               float* x, void* stream) {
  using namespace kdlae;
  if (!frames || !x || B <= 0 || F <= 0 || h <= 0 || w <= 0 || multiple <= 0) return fail(KDLAE_ESTATE, "bad argument");
  if (channels != 1 && channels != 3 && channels != 4) return fail(KDLAE_EINVAL_SHAPE, "channels must be 1, 3 or 4");
  int H, W;
  kdlae_padded_size(h, w, multiple, &H, &W);
  if (H - h >= h || W - w >= w) return fail(KDLAE_EINVAL_SHAPE, "frame smaller than its reflect padding");
  // the F frames of a sample are independent images: [B*F][h][w][channels] -> [B*F][1][H][W] = [B][F][H][W]
  PreParams p{frames, B * F, h, w, channels, 1, 0, 1, H, W, x, nullptr, nullptr};
  HIPCHK(launch_preprocess_u8(p, reinterpret_cast<hipStream_t>(stream)));
  return KDLAE_OK;
}

void kdlae_padded_size(int h, int w, int multiple, int* H, int* W) {
  // KDLAE_T.ipynb: H = ((h + m) // m) * m, padded only when h % m != 0
  *H = (h % multiple) ? (h + multiple) / multiple * multiple : h;
  *W = (w % multiple) ? (w + multiple) / multiple * multiple : w;
}

int kdlae_postprocess_u8(const float* out, int B, int C, int Hs, int Ws, int h, int w, int scale,
                         const uint8_t* lq, int lq_channels, uint8_t* dst, void* stream) {
  using namespace kdlae;
  if (!out || !dst || B <= 0 || h <= 0 || w <= 0) return fail(KDLAE_ESTATE, "bad argument");
  if (lq && lq_channels != 1 && lq_channels != 3 && lq_channels != 4)
    return fail(KDLAE_EINVAL_SHAPE, "lq_channels must be 1, 3 or 4");
  PostParams p{out, B, C, Hs, Ws, h, w, scale, lq, lq_channels, dst};
  HIPCHK(launch_postprocess_u8(p, reinterpret_cast<hipStream_t>(stream)));
  return KDLAE_OK;
}

}  // extern "C"
