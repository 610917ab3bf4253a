// Accuracy probe of the hardware sine / cosine against libm in double (profiling aid, not a product path):
//   hipcc -O3 --offload-arch=gfx950 -o tools/_probe/trig_probe tools/trig_probe.hip && tools/_probe/trig_probe
// x on [-pi, pi] (joint angles) and [-0.6, 0.6] (a substep's half rotation); the argument in revolutions, reduced
// to [-1/2, 1/2], as the kernels would pass it (device_math.hpp psincos); also the library's sinf / cosf on device.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k_trig(const float* x, float* s, float* c, float* ls, float* lc, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float r = x[i] * 0.159154943091895336f;
  r = r - __builtin_rintf(r);
  s[i] = __builtin_amdgcn_sinf(r);
  c[i] = __builtin_amdgcn_cosf(r);
  ls[i] = sinf(x[i]);
  lc[i] = cosf(x[i]);
}

int main() {
  const int n = 1 << 22;
  for (double range : {3.14159265358979, 0.6}) {
    std::vector<float> x(n), s(n), c(n), ls(n), lc(n);
    for (int i = 0; i < n; i++) x[i] = (float)(range * (2.0 * (i + 0.5) / n - 1.0));
    float *dx, *ds, *dc, *dls, *dlc;
    hipMalloc(&dx, n * 4); hipMalloc(&ds, n * 4); hipMalloc(&dc, n * 4); hipMalloc(&dls, n * 4); hipMalloc(&dlc, n * 4);
    hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_trig, dim3((n + 255) / 256), dim3(256), 0, 0, dx, ds, dc, dls, dlc, n);
    hipMemcpy(s.data(), ds, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(ls.data(), dls, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(lc.data(), dlc, n * 4, hipMemcpyDeviceToHost);
    double hs = 0, hc = 0, lsm = 0, lcm = 0, hrs = 0;
    for (int i = 0; i < n; i++) {
      const double S = std::sin((double)x[i]), C = std::cos((double)x[i]);
      hs = std::fmax(hs, std::fabs(s[i] - S)); hc = std::fmax(hc, std::fabs(c[i] - C));
      lsm = std::fmax(lsm, std::fabs(ls[i] - S)); lcm = std::fmax(lcm, std::fabs(lc[i] - C));
      if (std::fabs(S) > 1e-3) hrs = std::fmax(hrs, std::fabs(s[i] - S) / std::fabs(S));
    }
    printf("|x| <= %.3f: hardware max abs err sin %.3g cos %.3g (sin rel, |sin| > 1e-3: %.3g); library sinf %.3g cosf %.3g\n",
           range, hs, hc, hrs, lsm, lcm);
    hipFree(dx); hipFree(ds); hipFree(dc); hipFree(dls); hipFree(dlc);
  }
  return 0;
}
