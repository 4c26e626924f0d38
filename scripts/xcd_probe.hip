// Probe: does the dispatcher keep "blocks b and b + 8 share an XCD" for a large grid of short
// blocks that run many waves deep (the metric item kernel's launch shape)?  Each block does a
// little gather work (so blocks retire at different times) and lane 0 of wave 0 records the XCD it
// ran on (HW_REG_XCC_ID) with a plain vector store.  The host counts, for every label b % 8, how
// many of its blocks ran on that label's most common XCD.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/xcd_probe scripts/xcd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) k_probe(const float* __restrict__ x, int n, int* __restrict__ xcc,
                                               float* __restrict__ sink) {
  const int lane = threadIdx.x;
  // a few dependent gathers of varying length per block
  float acc = 0.f;
  unsigned h = blockIdx.x * 2654435761u + lane;
  const int len = 4 + (blockIdx.x * 7919u) % 29;
  for (int i = 0; i < len; ++i) {
    h = h * 1664525u + 1013904223u;
    acc += x[h % static_cast<unsigned>(n)];
  }
  if (lane == 0) {
    const unsigned id = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
    xcc[blockIdx.x] = static_cast<int>(id & 15u);
  }
  if (acc == 12345.f) sink[lane] = acc;  // keep the loads
}

int main() {
  const int n = 1 << 24, blocks = 1 << 18;
  float *x = nullptr, *sink = nullptr;
  int* xcc = nullptr;
  if (hipMalloc(&x, n * sizeof(float)) || hipMalloc(&sink, 256 * sizeof(float)) ||
      hipMalloc(&xcc, blocks * sizeof(int)))
    return 1;
  hipMemset(x, 0, n * sizeof(float));
  hipMemset(xcc, 0xff, blocks * sizeof(int));
  k_probe<<<blocks, 256>>>(x, n, xcc, sink);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::vector<int> h(blocks);
  hipMemcpy(h.data(), xcc, blocks * sizeof(int), hipMemcpyDeviceToHost);
  long same = 0, total = 0;
  int hist[8][16] = {};
  for (int b = 0; b < blocks; ++b)
    if (h[b] >= 0 && h[b] < 16) hist[b % 8][h[b]]++;
  printf("{\"blocks\": %d, \"labels\": [", blocks);
  for (int l = 0; l < 8; ++l) {
    int best = 0, arg = 0, tot = 0;
    for (int c = 0; c < 16; ++c) {
      tot += hist[l][c];
      if (hist[l][c] > best) best = hist[l][c], arg = c;
    }
    same += best;
    total += tot;
    printf("%s{\"label\": %d, \"xcc\": %d, \"share\": %.4f}", l ? ", " : "", l, arg, tot ? double(best) / tot : 0.0);
  }
  printf("], \"same_xcd_fraction\": %.5f}\n", total ? double(same) / total : 0.0);
  hipFree(x);
  hipFree(sink);
  hipFree(xcc);
  return 0;
}
