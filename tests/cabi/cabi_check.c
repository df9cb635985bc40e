/* C caller of the C ABI (include/sdmi.h) without PyTorch: a 3x3 convolution as an implicit GEMM (sdmi_gemm_plan +
 * sdmi_gemm, the nn.Conv2d of models/blocks.py:48-53) and a cross-attention core (sdmi_attn_fwd, the
 * nn.MultiheadAttention core of models/blocks.py:140) on deterministic inputs. Writes every input and output as a
 * raw little-endian file into argv[1]; tests/test_cabi_gpu.py compares them with torch fp32. Built by
 * __graft_entry__.build() (gcc, HIP runtime + libsdmi.so). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#include "sdmi.h"

static uint32_t lcg_state = 12345u;
static float frand(void) { /* uniform in [-1, 1) */
  lcg_state = lcg_state * 1664525u + 1013904223u;
  return (float)((lcg_state >> 8) & 0xFFFFFF) / 8388608.0f - 1.0f;
}
static uint16_t f2bf(float f) { /* round to nearest even */
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

#define CHECK_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 2; } } while (0)
#define CHECK_SDMI(x) do { int r_ = (x); if (r_ != 0) { fprintf(stderr, "%s returned %d\n", #x, r_); return 3; } } while (0)

static int dump(const char* dir, const char* name, const void* host, size_t bytes) {
  char path[1024];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(host, 1, bytes, f) != bytes) { fprintf(stderr, "cannot write %s\n", path); return 1; }
  fclose(f);
  return 0;
}

static int upload_bf16(size_t n, float scale, uint16_t** host, void** dev) {
  *host = (uint16_t*)malloc(n * 2);
  for (size_t i = 0; i < n; ++i) (*host)[i] = f2bf(frand() * scale);
  if (hipMalloc(dev, n * 2) != hipSuccess) return 1;
  return hipMemcpy(*dev, *host, n * 2, hipMemcpyHostToDevice) != hipSuccess;
}

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s OUT_DIR\n", argv[0]); return 1; }
  const char* dir = argv[1];
  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));

  /* ---- conv 3x3, stride 1, padding 1: x NHWC bf16 [B][H][W][Cin], w packed [Cout][3][3][Cin], fp32 bias ---- */
  const int B = 2, H = 16, W = 16, Cin = 64, Cout = 128;
  uint16_t *hx, *hw;
  void *dx, *dw, *dy, *db, *dws = NULL;
  if (upload_bf16((size_t)B * H * W * Cin, 1.0f, &hx, &dx)) return 2;
  if (upload_bf16((size_t)Cout * 9 * Cin, 0.05f, &hw, &dw)) return 2;
  float* hb = (float*)malloc(Cout * 4);
  for (int i = 0; i < Cout; ++i) hb[i] = frand() * 0.1f;
  CHECK_HIP(hipMalloc(&db, Cout * 4));
  CHECK_HIP(hipMemcpy(db, hb, Cout * 4, hipMemcpyHostToDevice));
  CHECK_HIP(hipMalloc(&dy, (size_t)B * H * W * Cout * 2));
  sdmi_gemm_desc d;
  memset(&d, 0, sizeof d);
  d.m = B * H * W; d.n = Cout; d.k = 9 * Cin;
  d.a_mode = SDMI_A_CONV; d.a = dx;
  /* ih, iw, cin, ldx, kh, kw, oh, ow (the GEMM pixel grid), sy, sx, oy0, ox0 */
  sdmi_conv_geom g = {H, W, Cin, Cin, 3, 3, H, W, 1, 1, -1, -1};
  d.geom = g;
  d.b_mode = SDMI_B_NK; d.b = dw; d.ldb = 9 * Cin;
  d.c = dy; d.ldc = Cout; d.bias = (const float*)db; d.alpha = 1.0f;
  int splits = 0;
  size_t ws = 0;
  CHECK_SDMI(sdmi_gemm_plan(&d, &splits, &ws));
  if (ws) CHECK_HIP(hipMalloc(&dws, ws));
  CHECK_SDMI(sdmi_gemm(&d, dws, ws, stream));

  /* ---- attention core: q [B*N][C], k / v [B*S][C], heads of d = C / heads ---- */
  const int N = 256, S = 77, heads = 4, hd = 32, C = heads * hd;
  uint16_t *hq, *hk, *hv;
  void *dq, *dk, *dv, *dout, *dlse;
  if (upload_bf16((size_t)B * N * C, 1.0f, &hq, &dq)) return 2;
  if (upload_bf16((size_t)B * S * C, 1.0f, &hk, &dk)) return 2;
  if (upload_bf16((size_t)B * S * C, 1.0f, &hv, &dv)) return 2;
  CHECK_HIP(hipMalloc(&dout, (size_t)B * N * C * 2));
  CHECK_HIP(hipMalloc(&dlse, (size_t)B * heads * N * 4));
  CHECK_SDMI(sdmi_attn_fwd(dq, C, dk, C, dv, C, dout, C, (float*)dlse, B, heads, N, S, hd, stream));
  CHECK_HIP(hipStreamSynchronize(stream));

  size_t ny = (size_t)B * H * W * Cout, no = (size_t)B * N * C;
  uint16_t* hy = (uint16_t*)malloc(ny * 2);
  uint16_t* ho = (uint16_t*)malloc(no * 2);
  float* hl = (float*)malloc((size_t)B * heads * N * 4);
  CHECK_HIP(hipMemcpy(hy, dy, ny * 2, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(ho, dout, no * 2, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(hl, dlse, (size_t)B * heads * N * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  bad |= dump(dir, "conv_x.bf16", hx, (size_t)B * H * W * Cin * 2);
  bad |= dump(dir, "conv_w.bf16", hw, (size_t)Cout * 9 * Cin * 2);
  bad |= dump(dir, "conv_b.f32", hb, Cout * 4);
  bad |= dump(dir, "conv_y.bf16", hy, ny * 2);
  bad |= dump(dir, "attn_q.bf16", hq, no * 2);
  bad |= dump(dir, "attn_k.bf16", hk, (size_t)B * S * C * 2);
  bad |= dump(dir, "attn_v.bf16", hv, (size_t)B * S * C * 2);
  bad |= dump(dir, "attn_o.bf16", ho, no * 2);
  bad |= dump(dir, "attn_lse.f32", hl, (size_t)B * heads * N * 4);
  printf("cabi_check: conv splits=%d ws=%zu, attention done\n", splits, ws);
  return bad;
}
