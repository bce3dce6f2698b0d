// Device-side helpers shared by the gfx950 kernel translation units.
#pragma once
#include <hip/hip_runtime.h>

namespace vox {

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// Ragged batches (vox_embed_device_lens): utterance n of a batch padded to H
// rows holds vlen[n] frames.  At a layer downsampled by 2^vsh its valid rows are
// ceil(vlen[n] / 2^vsh) -- every stride-2 layer (TF fixed padding / SAME, k = 3)
// maps an input of h rows to ceil(h / 2) -- and a kernel reads the rows at or
// past that as the zero padding of an utterance ending there, so a padded
// utterance's valid outputs equal the unpadded run's.  vlen null: H.
__device__ __forceinline__ int valid_rows(const int* vlen, int vsh, int n, int H) {
  return vlen ? min(H, (vlen[n] + (1 << vsh) - 1) >> vsh) : H;
}

// TF1 nn.batch_normalization at inference (the 2-D head BNs, non-fused):
// x * inv + (-mean * inv) as two roundings -- its Mul and Add graph ops --
// never contracted to an FMA; nmi = -mean * inv is precomputed at load
__device__ __forceinline__ float bn2d(float x, float inv, float nmi) {
#pragma clang fp contract(off)
  return x * inv + nmi;
}

__device__ __forceinline__ bf16x8 ld16(const bf16_t* p) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  return __builtin_bit_cast(bf16x8, u);
}
__device__ __forceinline__ f32x4 ld16(const float* p) {
  return *reinterpret_cast<const f32x4*>(p);
}

template <typename F> __device__ __forceinline__ F zero_frag() { return F{}; }

// Elementwise helpers on fragments (in fp32).
__device__ __forceinline__ bf16x8 frag_add(bf16x8 a, bf16x8 b) {
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (bf16_t)((float)a[e] + (float)b[e]);
  return r;
}
__device__ __forceinline__ f32x4 frag_add(f32x4 a, f32x4 b) { return a + b; }

// ReLU on bf16 bit patterns: every negative value (and -0) has the sign bit
// set, i.e. is a negative int16, so a packed int16 max with 0 is ReLU.  bf16
// rounding is monotone and keeps the sign, so relu(bf16(x)) == bf16(relu(x))
// bit for bit; one v_pk_max_i16 per two channels instead of two v_max_f32.
__device__ __forceinline__ bf16x4 relu_bf16(bf16x4 v) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  const s16x4 s = __builtin_elementwise_max(__builtin_bit_cast(s16x4, v), (s16x4){0, 0, 0, 0});
  return __builtin_bit_cast(bf16x4, s);
}
__device__ __forceinline__ bf16x8 relu_bf16(bf16x8 v) {
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 s = __builtin_elementwise_max(__builtin_bit_cast(s16x8, v),
                                            (s16x8){0, 0, 0, 0, 0, 0, 0, 0});
  return __builtin_bit_cast(bf16x8, s);
}

// Global loads / stores issued as inline asm, for kernels that count their
// own vmcnt: the compiler's waitcnt pass cannot prove which older loads a later
// use depends on across role branches and falls back to vmcnt(0), which also
// waits for every store the wave has in flight.  A value loaded with vld16 is
// valid only after vm_wait(n) (n = this wave's vector-memory ops issued after
// it) and vm_launder(v) (so the compiler does not hoist uses above the wait).
// Soundness rule: on EVERY path from a vld16 the wave must reach a covering
// vm_wait followed by vm_launder of the destination before the variable is
// reassigned or the kernel ends.  The compiler does not know the load is in
// flight: where the value is dead on some path (never laundered there), it
// reuses the registers at once -- e.g. for the next loads' addresses -- and the
// late data then overwrites them (tools/vmcnt_audit.py checks the ISA).
// No "memory" clobbers: the kernels never read back what these touch, and a
// clobber would pin every LDS access around each store.
typedef unsigned vu32x4 __attribute__((ext_vector_type(4)));
// The load itself is an ordinary (compiler-visible) global load: the
// compiler's waitcnt pass then covers every use and every register copy of the
// destination, so no allocation choice can let a late load land in a register
// that holds something else (an inline-asm load whose destination the
// compiler believes written at issue was copied into the loop-carried
// prefetch buffer before the data arrived in one build -- tools/vmcnt_audit.py).
// The asm stores below are invisible to that pass, which only makes its
// counts conservative (it waits for them too), never unsafe; vm_wait /
// vm_launder keep marking where the kernels expect each load to have landed.
__device__ __forceinline__ void vld16(vu32x4& v, const void* p) {
  v = *reinterpret_cast<const vu32x4*>(p);
}
// the trailing s_nop keeps the next instruction from overwriting the data
// registers before the store has read them
__device__ __forceinline__ void vst16(void* p, vu32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" : : "v"(p), "v"(v));
}
template <typename T>
__device__ __forceinline__ void vm_launder(T& v) {
  asm volatile("" : "+v"(v));
}
#define VOX_VMW(n) \
  case n: asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory"); break;
// s_waitcnt vmcnt(n) for a wave-uniform n (a scalar branch to the immediate form)
__device__ __forceinline__ void vm_wait(int n) {
  switch (n) {
    VOX_VMW(0) VOX_VMW(1) VOX_VMW(2) VOX_VMW(3) VOX_VMW(4) VOX_VMW(5) VOX_VMW(6) VOX_VMW(7)
    VOX_VMW(8) VOX_VMW(9) VOX_VMW(10) VOX_VMW(11) VOX_VMW(12) VOX_VMW(13) VOX_VMW(14)
    VOX_VMW(15) VOX_VMW(16) VOX_VMW(17) VOX_VMW(18) VOX_VMW(19) VOX_VMW(20) VOX_VMW(21)
    VOX_VMW(22) VOX_VMW(23) VOX_VMW(24) VOX_VMW(25) VOX_VMW(26) VOX_VMW(27) VOX_VMW(28)
    VOX_VMW(29) VOX_VMW(30) VOX_VMW(31) VOX_VMW(32) VOX_VMW(33) VOX_VMW(34) VOX_VMW(35)
    VOX_VMW(36) VOX_VMW(37) VOX_VMW(38) VOX_VMW(39) VOX_VMW(40)
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
  __builtin_amdgcn_sched_barrier(0);
}
#undef VOX_VMW

__device__ __forceinline__ f32x4 mfma_step(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

}  // namespace vox
