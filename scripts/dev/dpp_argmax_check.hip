#include <hip/hip_runtime.h>
__device__ __forceinline__ float dpp_f(float v, int ctrl_dummy);
template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(v, v, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ void amax_step(float& v, int& i, float v2, int i2) {
  if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void wave_argmax_dpp(float& v, int& i) {
  amax_step(v, i, dppf<0xB1>(v), dppi<0xB1>(i));
  amax_step(v, i, dppf<0x4E>(v), dppi<0x4E>(i));
  amax_step(v, i, dppf<0x124>(v), dppi<0x124>(i));
  amax_step(v, i, dppf<0x128>(v), dppi<0x128>(i));
  float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
  int ri = __builtin_amdgcn_readlane(i, 0);
  #pragma unroll
  for (int l = 16; l < 64; l += 16) {
    float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
    int i2 = __builtin_amdgcn_readlane(i, l);
    amax_step(r, ri, r2, i2);
  }
  v = r; i = ri;
}
__global__ void k(const float* x, float* outv, int* outi) {
  float v = x[blockIdx.x * 64 + threadIdx.x];
  int i = threadIdx.x;
  wave_argmax_dpp(v, i);
  outv[blockIdx.x * 64 + threadIdx.x] = v;
  outi[blockIdx.x * 64 + threadIdx.x] = i;
}
int main() {
  const int B = 1000;
  float* hx = new float[B * 64];
  srand(1);
  for (int j = 0; j < B * 64; ++j) hx[j] = (float)(rand() % 50);
  float *dx, *dv; int* di;
  hipMalloc(&dx, B * 64 * 4); hipMalloc(&dv, B * 64 * 4); hipMalloc(&di, B * 64 * 4);
  hipMemcpy(dx, hx, B * 64 * 4, hipMemcpyHostToDevice);
  k<<<B, 64>>>(dx, dv, di);
  float* hv = new float[B * 64]; int* hi = new int[B * 64];
  hipMemcpy(hv, dv, B * 64 * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hi, di, B * 64 * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int b = 0; b < B; ++b) {
    float m = -1; int mi = 0;
    for (int l = 0; l < 64; ++l) if (hx[b * 64 + l] > m) { m = hx[b * 64 + l]; mi = l; }
    for (int l = 0; l < 64; ++l) if (hv[b * 64 + l] != m || hi[b * 64 + l] != mi) ++bad;
  }
  printf("bad %d\n", bad);
  return bad != 0;
}
