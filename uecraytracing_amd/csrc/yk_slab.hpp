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
// Two slots' near / far distances in one asm block (YK_CULL_BLOCK): tn = max(max3(near), tmin),
// tf = min(min3(far), ustar) for slots a and b, interleaved so that no instruction reads a result
// of the one before it.  The same eight instructions as four slab_max3 / slab_max / slab_min3 /
// slab_min pairs; one block instead of eight lets the hazard recognizer, which cannot see into an
// asm block, pad only its edges.
__device__ __forceinline__ void slab_cull2(float na0, float na1, float na2, float fa0, float fa1, float fa2,
                                           float nb0, float nb1, float nb2, float fb0, float fb1, float fb2,
                                           float tmin, float ustar, float& tna, float& tfa, float& tnb,
                                           float& tfb) {
  asm("v_max3_f32 %0, %6, %7, %8\n\t"
      "v_max3_f32 %2, %12, %13, %14\n\t"
      "v_min3_f32 %1, %9, %10, %11\n\t"
      "v_min3_f32 %3, %15, %16, %17\n\t"
      "v_max_f32 %0, %0, %4\n\t"
      "v_max_f32 %2, %2, %4\n\t"
      "v_min_f32 %1, %1, %5\n\t"
      "v_min_f32 %3, %3, %5"
      : "=&v"(tna), "=&v"(tfa), "=&v"(tnb), "=&v"(tfb)
      : "v"(tmin), "v"(ustar), "v"(na0), "v"(na1), "v"(na2), "v"(fa0), "v"(fa1), "v"(fa2), "v"(nb0), "v"(nb1),
        "v"(nb2), "v"(fb0), "v"(fb1), "v"(fb2));
}
// slab_fma with the clamp modifier (YK_NEAR_CLAMP): both results clamped to [0, 1]
__device__ __forceinline__ f2 slab_fma_clamp(f2 plane, f2 p) {
  f2 r;
  asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1] clamp" : "=v"(r) : "v"(plane), "v"(p));
  return r;
}
// slab_cull2 for clamped near distances (YK_NEAR_CLAMP): tn = max3(near) (the clamp was the max
// with the lower bound), tf = min(min3(far), ustar)
__device__ __forceinline__ void slab_cull2c(float na0, float na1, float na2, float fa0, float fa1, float fa2,
                                            float nb0, float nb1, float nb2, float fb0, float fb1, float fb2,
                                            float ustar, float& tna, float& tfa, float& tnb, float& tfb) {
  asm("v_min3_f32 %1, %8, %9, %10\n\t"
      "v_min3_f32 %3, %14, %15, %16\n\t"
      "v_max3_f32 %0, %5, %6, %7\n\t"
      "v_max3_f32 %2, %11, %12, %13\n\t"
      "v_min_f32 %1, %1, %4\n\t"
      "v_min_f32 %3, %3, %4"
      : "=&v"(tna), "=&v"(tfa), "=&v"(tnb), "=&v"(tfb)
      : "v"(ustar), "v"(na0), "v"(na1), "v"(na2), "v"(fa0), "v"(fa1), "v"(fa2), "v"(nb0), "v"(nb1), "v"(nb2),
        "v"(fb0), "v"(fb1), "v"(fb2));
}
