// Gradient routing of the ResNet stem max-pool (3x3, stride 2, pad 1) backward, shared by the
// pool backward (pool.hip maxpool_bwd_s2_kernel) and the fused stem BN backward
// (batchnorm.hip stem_pool_bwd_apply_kernel): the 2x2 input pixels (2i .. 2i+1, 2j .. 2j+1) of
// output position (i, j) collect the gradient of every window whose stored argmax (uint8 window
// offset kh * 3 + kw) is one of them — windows (i, j), (i, j+1), (i+1, j), (i+1, j+1) — in a fixed
// order (deterministic).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ndp {

__device__ __forceinline__ void pool_s2_route(const float* __restrict__ dyp, const uint8_t* __restrict__ ip, int i,
                                              int j, int OH, int OW, float& d00, float& d01, float& d10,
                                              float& d11) {
  const bool right = j + 1 < OW, down = i + 1 < OH;
  const int c = i * OW + j;
  const float g00 = dyp[c], g01 = right ? dyp[c + 1] : 0.f, g10 = down ? dyp[c + OW] : 0.f,
              g11 = (right && down) ? dyp[c + OW + 1] : 0.f;
  const int a00 = ip[c], a01 = right ? ip[c + 1] : -1, a10 = down ? ip[c + OW] : -1,
            a11 = (right && down) ? ip[c + OW + 1] : -1;
  // window (oh, ow) covers input rows 2oh-1 .. 2oh+1: tap kh = h - 2oh + 1
  d00 = d01 = d10 = d11 = 0.f;
  if (a00 == 4) d00 += g00;                     // (2i, 2j)     <- (i, j) tap (1,1)
  if (a00 == 5) d01 += g00;                     // (2i, 2j+1)   <- (i, j) tap (1,2)
  if (a01 == 3) d01 += g01;                     //              <- (i, j+1) tap (1,0)
  if (a00 == 7) d10 += g00;                     // (2i+1, 2j)   <- (i, j) tap (2,1)
  if (a10 == 1) d10 += g10;                     //              <- (i+1, j) tap (0,1)
  if (a00 == 8) d11 += g00;                     // (2i+1, 2j+1) <- (i, j) tap (2,2)
  if (a01 == 6) d11 += g01;                     //              <- (i, j+1) tap (2,0)
  if (a10 == 2) d11 += g10;                     //              <- (i+1, j) tap (0,2)
  if (a11 == 0) d11 += g11;                     //              <- (i+1, j+1) tap (0,0)
}

// The same routing when the 64 lanes of a wave are one 8x8 pooled plane (lane = 8 i + j): each lane
// loads only its own dY / argmax and takes its right / lower / diagonal neighbours' by lane shuffle
// (4x fewer loads; the sums are the same, in the same order).
__device__ __forceinline__ void pool_s2_route_wave(float g00, int a00, int i, int j, float& d00, float& d01,
                                                   float& d10, float& d11) {
  const int lane = (int)(threadIdx.x & 63);
  const bool right = j + 1 < 8, down = i + 1 < 8;
  const float s01 = __shfl(g00, (lane + 1) & 63, 64), s10 = __shfl(g00, (lane + 8) & 63, 64),
              s11 = __shfl(g00, (lane + 9) & 63, 64);
  const int t01 = __shfl(a00, (lane + 1) & 63, 64), t10 = __shfl(a00, (lane + 8) & 63, 64),
            t11 = __shfl(a00, (lane + 9) & 63, 64);
  const float g01 = right ? s01 : 0.f, g10 = down ? s10 : 0.f, g11 = (right && down) ? s11 : 0.f;
  const int a01 = right ? t01 : -1, a10 = down ? t10 : -1, a11 = (right && down) ? t11 : -1;
  d00 = d01 = d10 = d11 = 0.f;
  if (a00 == 4) d00 += g00;
  if (a00 == 5) d01 += g00;
  if (a01 == 3) d01 += g01;
  if (a00 == 7) d10 += g00;
  if (a10 == 1) d10 += g10;
  if (a00 == 8) d11 += g00;
  if (a01 == 6) d11 += g01;
  if (a10 == 2) d11 += g10;
  if (a11 == 0) d11 += g11;
}

}  // namespace ndp
