// Probe: v_pk_add_f32 with op_sel / neg modifiers, destination distinct from / equal to a source.
// Build + run: hipcc --offload-arch=gfx950 -O3 tools/pk_probe.hip -o gpurun_out/pk_probe && gpurun_out/pk_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
__global__ void k(const float* in, float* out) {
  const int i = threadIdx.x;
  f2 a = {in[4 * i], in[4 * i + 1]}, b = {in[4 * i + 2], in[4 * i + 3]};
  f2 r[6];
  // form 1: (a.x - b.x, a.y + b.x); form 2: (-a.y + b.x, a.y - b.y)
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r[0]) : "v"(a), "v"(b));
  asm volatile("v_pk_add_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]" : "=v"(r[1]) : "v"(a), "v"(b));
  f2 a2 = a, b2 = b;
  asm volatile("v_pk_add_f32 %0, %0, %1 op_sel_hi:[1,0] neg_lo:[0,1]" : "+v"(a2) : "v"(b));  // dest = src0
  r[2] = a2;
  asm volatile("v_pk_add_f32 %0, %1, %0 op_sel_hi:[1,0] neg_lo:[0,1]" : "+v"(b2) : "v"(a));  // dest = src1
  r[3] = b2;
  a2 = a; b2 = b;
  asm volatile("v_pk_add_f32 %0, %0, %1 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]" : "+v"(a2) : "v"(b));
  r[4] = a2;
  asm volatile("v_pk_add_f32 %0, %1, %0 op_sel:[1,0] op_sel_hi:[1,1] neg_lo:[1,0] neg_hi:[0,1]" : "+v"(b2) : "v"(a));
  r[5] = b2;
  for (int j = 0; j < 6; ++j) { out[12 * i + 2 * j] = r[j].x; out[12 * i + 2 * j + 1] = r[j].y; }
}
int main() {
  float h[256], o[64 * 12];
  for (int i = 0; i < 256; ++i) h[i] = (float)(i * 7 % 31) + 0.25f * (i % 3);
  float *di, *dout;
  hipMalloc(&di, sizeof(h)); hipMalloc(&dout, sizeof(o));
  hipMemcpy(di, h, sizeof(h), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, di, dout);
  hipMemcpy(o, dout, sizeof(o), hipMemcpyDeviceToHost);
  int bad[6] = {0};
  for (int i = 0; i < 64; ++i) {
    const float ax = h[4 * i], ay = h[4 * i + 1], bx = h[4 * i + 2], by = h[4 * i + 3];
    const float e1[2] = {ax - bx, ay + bx}, e2[2] = {-ay + bx, ay - by};
    for (int j = 0; j < 6; ++j) {
      const float* e = (j == 0 || j == 2 || j == 3) ? e1 : e2;
      if (o[12 * i + 2 * j] != e[0] || o[12 * i + 2 * j + 1] != e[1]) {
        if (bad[j]++ == 0)
          printf("form %d lane %d: got (%g, %g) want (%g, %g)  a=(%g,%g) b=(%g,%g)\n", j, i, o[12 * i + 2 * j],
                 o[12 * i + 2 * j + 1], e[0], e[1], ax, ay, bx, by);
      }
    }
  }
  printf("bad per form (distinct f1, distinct f2, f1 dst=a, f1 dst=b, f2 dst=a, f2 dst=b): %d %d %d %d %d %d\n", bad[0],
         bad[1], bad[2], bad[3], bad[4], bad[5]);
  return 0;
}
