// yk_slab.hpp — the wide-node slab test's arithmetic in the fewest registers (gfx950; included by
// ykgpu_render.hip inside its anonymous namespace).
//
// d = plane * p.x + p.y for both slots of a plane pair, the pair (1/d, -o/d) read by op_sel: one
// v_pk_fma_f32 whose second and third operands are the two halves of ONE register pair (the
// compiler would keep each broadcast operand as a register pair of its own).  The slab min/max
// below are asm too: an asm result is not known to be canonical, and the compiler would otherwise
// quiet it with an extra v_max before every fmaxf/fminf.  Same instructions, same rounding as
// the compiler's fmaxf / fminf chains of the visit.
__device__ __forceinline__ f2 slab_fma(f2 plane, f2 p) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(plane), "v"(p));
  return r;
}
__device__ __forceinline__ float slab_max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float slab_min3(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float slab_max(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float slab_min(float a, float b) {
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
