// Host-only probe: the ctx / workspace layouts a source tree's planners give one descriptor with the module
// path's NCHW flag off (query / prologue time) and on (launch time).  Build against any revision's csrc:
//   hipcc -O1 -std=c++17 -I<tree>/cim_quantization_amd/csrc tools/layout_probe.cpp -o /tmp/layout_probe
// (the round-5 first-visit fault)
#include "cimq_host.h"

int main() {
  using namespace cimq;
  // bench.RESNET20's distinct w3a3 shapes: (C, O, H, stride)
  const int shapes[][4] = {{16, 16, 32, 1}, {16, 32, 32, 2}, {32, 32, 16, 1}, {32, 64, 16, 2}, {64, 64, 8, 1}};
  for (auto& s : shapes) {
    cimq_conv_desc d;
    memset(&d, 0, sizeof(d));
    d.batch = 256; d.in_channels = s[0]; d.in_h = d.in_w = s[2]; d.out_channels = s[1];
    d.kernel_h = d.kernel_w = 3; d.stride_h = d.stride_w = s[3]; d.pad_h = d.pad_w = 1; d.xbar = 128;
    d.bits_w = d.bits_a = 3; d.bs_w = d.bs_a = 1; d.adc_bits = 1.5f; d.input_kind = CIMQ_INPUT_RAW_LSQ; d.lsq_qp = 7.f;
    Geo g;
    if (make_geo(&d, &g) != 0) { printf("make_geo failed\n"); return 1; }
    size_t ct[2], wt[2], st[2];
    for (int n = 0; n < 2; ++n) {
      g.onchw = n;
      const CtxLayout L = ctx_layout(g);
      const WsLayout W = ws_layout(g);
      ct[n] = L.total; st[n] = L.st; wt[n] = W.total;
    }
    printf("C%-3d O%-3d H%-3d s%d  ctx %zu -> %zu (st at %zu -> %zu)  ws %zu -> %zu\n", s[0], s[1], s[2], s[3], ct[0], ct[1],
           st[0], st[1], wt[0], wt[1]);
  }
  return 0;
}
