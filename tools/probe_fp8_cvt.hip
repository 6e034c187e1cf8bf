// Probe of gfx950's fp8 conversion instructions on edge values: NaN, +-inf,
// past-max magnitudes, raw and after a v_med3_f32 clamp to max finite, and
// v_med3_f32's NaN behaviour.  Prints one line per input value.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

__global__ void k(const float* x, int n, unsigned* out) {
  int i = threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  int a = __builtin_amdgcn_cvt_pk_fp8_f32(v, v, 0, false);
  int b = __builtin_amdgcn_cvt_pk_bf8_f32(v, v, 0, false);
  float mb = __builtin_amdgcn_fmed3f(v, -57344.0f, 57344.0f);
  int c = __builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(v, -448.0f, 448.0f), v, 0, false);
  int d = __builtin_amdgcn_cvt_pk_bf8_f32(mb, mb, 0, false);
  float m = __builtin_amdgcn_fmed3f(v, -448.0f, 448.0f);
  out[i * 5 + 0] = a & 0xff;
  out[i * 5 + 1] = b & 0xff;
  out[i * 5 + 2] = c & 0xff;
  out[i * 5 + 3] = d & 0xff;
  out[i * 5 + 4] = __float_as_uint(m);
}

int main() {
  float h[] = {NAN, -NAN, INFINITY, -INFINITY, 448.f, 464.f, 480.f, 1e6f, -1e6f, 57344.f, 61440.f,
               65536.f, -70000.f, 1.f, 0.001f, 1e-9f, -0.f};
  int n = sizeof(h) / sizeof(h[0]);
  float* dx; unsigned* dout;
  hipMalloc(&dx, sizeof(h)); hipMalloc(&dout, n * 5 * 4);
  hipMemcpy(dx, h, sizeof(h), hipMemcpyHostToDevice);
  k<<<1, 64>>>(dx, n, dout);
  unsigned o[17 * 5];
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  for (int i = 0; i < n; i++)
    printf("x=%-12g fp8=%02x bf8=%02x fp8_med3=%02x bf8_med3=%02x med3=%08x\n", h[i], o[i * 5],
           o[i * 5 + 1], o[i * 5 + 2], o[i * 5 + 3], o[i * 5 + 4]);
  return 0;
}
