// Device helpers shared by the gfx950 kernel files: LDS-DMA issue, counted
// vmcnt / lgkmcnt waits and barriers, hand-scheduled LDS accesses.
#pragma once
#include "asr_common.h"


namespace asr {
namespace blk {

static __device__ __attribute__((aligned(16))) uint4 g_zero_page[256];  // 4 KiB of zeros (DMA source for padding: one whole C=64 row)

typedef const __attribute__((address_space(1))) void* gptr_t;
typedef __attribute__((address_space(3))) void* lptr_t;

// One 1 KiB LDS-DMA (16 B per lane, lane-linear at the LDS address).  Inline
// asm, not the builtin: the compiler would otherwise wait vmcnt(0) before
// every later LDS read of the wave (it cannot tell the DMA's destination
// apart), serialising the prefetch with the compute.  Every reader of DMA'd
// data waits with a counted barrier_vm / vm_wait instead.  M0 is declared
// clobbered: the compiler re-establishes it only where it uses it (saving and
// restoring it around every DMA measured 0.7 % slower).
__device__ __forceinline__ void dma16(const void* src, unsigned char* lds_wave_base) {
  const unsigned l = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((ASR_LDS unsigned char*)lds_wave_base));
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "s"(l)
      : "memory", "m0");
}

// dma16 with the wave-uniform LDS byte address given directly (no generic ->
// LDS pointer conversion, whose null check trips a ROCm 7.2 codegen bug in
// register-tight kernels)
__device__ __forceinline__ void dma16_at(const void* src, unsigned lds_addr) {
  const unsigned l = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off"
      :
      : "v"(src), "s"(l)
      : "memory", "m0");
}

// Four consecutive 1 KiB LDS-DMA pieces on ONE address: the instruction offset
// advances the global source and the LDS destination alike (probed on gfx950,
// tools/probe/lds_dma_offset.hip), so a whole 4 KiB tile row costs one M0 write
// and no per-piece scalar address math.  (The per-piece form cost the
// stacked backward's wgrad waves ~1.8k cycles per band in scalar issue: 8
// waves' address arithmetic through one SALU slot per SIMD.)
__device__ __forceinline__ void dma16x4_at(const void* src, unsigned lds_addr) {
  const unsigned l = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile(
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %0, off\n\t"
      "global_load_lds_dwordx4 %0, off offset:1024\n\t"
      "global_load_lds_dwordx4 %0, off offset:2048\n\t"
      "global_load_lds_dwordx4 %0, off offset:3072"
      :
      : "v"(src), "s"(l)
      : "memory", "m0");
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
// 16-B / 4-B global loads the compiler does not track: it inserts no wait
// before their results are used.  For operands reloaded inside a loop whose
// next iteration starts with a counted barrier_vm that retires them (every
// vector-memory op older than the stores issued after them): with tracked
// loads hipcc waits vmcnt(0) before the first use, which also waits for the
// LDS-DMA of the next band issued since.  "+v": the result lands in the
// registers the value already lives in (tests/test_isa.py checks that no
// instruction reads them before the wait).
// Wave-uniform base (SGPRs) + 32-bit lane offset + immediate (< 4 KiB).  The
// base usually comes from v_readfirstlane (a VALU write of an SGPR), which a
// VMEM instruction may read only 5 wait states later; hipcc does not insert
// them in front of inline asm, so the asm does (s_nop 4).
template <int IMM, bool NOP = true>
__device__ __forceinline__ void gload128_untracked(u32x4& v, const void* sbase, unsigned voff) {
  static_assert(IMM >= 0 && IMM < 4096, "global immediate offset range");
  if constexpr (NOP)
    asm volatile("s_nop 4\n\tglobal_load_dwordx4 %0, %1, %2 offset:%3" : "+v"(v) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
  else  // (a later load of a run on the same base: the base's SGPR write is >= 5 states old)
    asm volatile("global_load_dwordx4 %0, %1, %2 offset:%3" : "+v"(v) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}
template <int IMM>
__device__ __forceinline__ void gload32_untracked(float& v, const void* sbase, unsigned voff) {
  static_assert(IMM >= 0 && IMM < 4096, "global immediate offset range");
  asm volatile("s_nop 4\n\tglobal_load_dword %0, %1, %2 offset:%3" : "+v"(v) : "v"(voff), "s"(sbase), "i"(IMM) : "memory");
}
// a pointer made wave-uniform (SGPRs)
__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const unsigned long long a = (unsigned long long)(uintptr_t)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return (const void*)(uintptr_t)(((unsigned long long)hi << 32) | lo);
}

// barrier for LDS data only (in-flight DMA and stores keep flying)
__device__ __forceinline__ void barrier_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ unsigned lds_u32(const void* p) {
  return (unsigned)(uintptr_t)((ASR_LDS const unsigned char*)p);
}

// Hand-scheduled LDS reads (hipcc would otherwise wait lgkmcnt(0) on the
// just-issued prefetch): "=v" output + explicit counted wait +
// sched_barrier (cdna_hip_programming.md §5.7, rule 18).
template <int OFF>
__device__ __forceinline__ bf16x8 ds_read128(unsigned addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// LDS accesses the compiler must not order behind in-flight LDS-DMA: hipcc
// waits vmcnt(0) before any plain LDS access while a global_load_lds is
// outstanding (it cannot tell the DMA's destination buffer apart), which
// would serialise the next band's prefetch with this band's work.  The
// caller waits lgkmcnt itself (lgkm_wait) before using a read result.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u32x4 lds_rd128(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ u32x2 lds_rd64(unsigned addr) {
  u32x2 v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ unsigned lds_rd_u8(unsigned addr) {
  unsigned v;
  asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
__device__ __forceinline__ void lds_wr128(unsigned addr, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(v) : "memory");
}

// Wait until at most n of this wave's vector-memory ops are outstanding
// (vmcnt retires in issue order): used for LDS-DMA'd data the compiler does
// not track.  n above 24 waits for more than needed, which stays correct.
__device__ __forceinline__ void vm_wait(int n) {
#define ASR_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (__builtin_amdgcn_readfirstlane(n)) {
    ASR_VMW(1) ASR_VMW(2) ASR_VMW(3) ASR_VMW(4) ASR_VMW(5) ASR_VMW(6) ASR_VMW(7) ASR_VMW(8)
    ASR_VMW(9) ASR_VMW(10) ASR_VMW(11) ASR_VMW(12) ASR_VMW(13) ASR_VMW(14) ASR_VMW(15) ASR_VMW(16)
    ASR_VMW(17) ASR_VMW(18) ASR_VMW(19) ASR_VMW(20) ASR_VMW(21) ASR_VMW(22) ASR_VMW(23) ASR_VMW(24)
    default:
      if (n > 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");  // waits for more: still correct
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      break;
  }
#undef ASR_VMW
}
// Workgroup barrier that waits only for this wave's vector-memory ops OLDER
// than its `n` youngest (vmcnt counts loads, stores and LDS-DMA in issue
// order).  Used so that the barrier guarding an LDS-DMA'd buffer does not
// also wait for the global stores issued after that DMA.
__device__ __forceinline__ void barrier_vm(int n) {
  vm_wait(n);  // the counted wait, then one barrier every path reaches
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// barrier_vm for a count that is usually K: the general vm_wait is a switch
// over 25 immediates, which hipcc lowers to a chain of predicate tests (~40
// scalar instructions and ~14 branches per call, r05f instruction mix): the
// usual count takes one compare and one wait instead
template <int K>
__device__ __forceinline__ void barrier_vm_usual(int n) {
  if (__builtin_amdgcn_readfirstlane(n) == K)
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(K) : "memory");
  else
    vm_wait(n);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// instructions one wave issues in a `for (j = wave; j < total; j += nw)` loop
__device__ __forceinline__ int strided_count(int total, int wave, int nw) {
  return total > wave ? (total - wave + nw - 1) / nw : 0;
}

// compiler-visible 16-B LDS load / store at an LDS byte address (integer -> LDS
// pointer, no generic cast): hipcc places the lgkmcnt waits itself, so spilling
// or copying the result is safe
__device__ __forceinline__ u32x4 lds_ld128(unsigned a) {
  return *(const __attribute__((address_space(3))) u32x4*)(size_t)a;
}
__device__ __forceinline__ void lds_st128(unsigned a, u32x4 v) {
  *(__attribute__((address_space(3))) u32x4*)(size_t)a = v;
}

// tr_pair from LDS byte addresses (+ a compile-time offset the compiler folds
// into the instruction's offset field); integer -> LDS pointer, no generic cast
template <int OFF>
__device__ __forceinline__ bf16x8 tr_pair_at(unsigned a0, unsigned a1) {
  typedef __attribute__((address_space(3))) s16x4* lp;
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(size_t)(a0 + OFF));
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lp)(size_t)(a1 + OFF));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return *(bf16x8*)&c;
}
// the same for the C=64 wgrad operands: the second half 16 pixels (2 KiB of a
// swizzled tile row: the XOR swizzle repeats every 8 pixels) after the first,
// both as immediate offsets on one address register
template <int OFF>
__device__ __forceinline__ bf16x8 tr_pair_px(unsigned a) {
  return tr_pair_at<OFF>(a, a + 2048u);
}
__device__ __forceinline__ bf16x8 tr_pair(const unsigned char* p0, const unsigned char* p1) {
  const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ASR_LDS s16x4*)p0);
  const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((ASR_LDS s16x4*)p1);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  s16x8 c = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return *(bf16x8*)&c;
}


// ---- epilogue helpers shared by the C=16 deep stack and the C=64 band kernels ----

// The two pixel tiles' accumulators of one output row (D layout: lane (lx, g)
// holds channels 4g..4g+3 of pixels lx and 16+lx) regrouped so that lane
// (lx, g) holds channels 8(g>>1) + i, i = 0..7, of pixel lx + 16(g&1)
// (v_permlane16_swap: odd rows of the first operand <-> even rows of the second).
__device__ __forceinline__ void regroup(const f32x4& c0, const f32x4& c1, float (&z)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(c0[e]), __float_as_uint(c1[e]), false, false);
    z[e] = __uint_as_float(s[0]);
    z[4 + e] = __uint_as_float(s[1]);
  }
}
__device__ __forceinline__ float lo_f(unsigned w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float hi_f(unsigned w) { return __uint_as_float(w & 0xffff0000u); }
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
// (a, b) * s + (c, d) on one v_pk_fma_f32
__device__ __forceinline__ f32x2 pk_fma(float s, f32x2 ab, f32x2 cd) {
  return __builtin_elementwise_fma((f32x2){s, s}, ab, cd);
}
// 1 if v > 0 else 0 (v_med3_i32; in asm so that the compiler does not turn the
// following shift into a compare + select per bit)
__device__ __forceinline__ unsigned bit01(int v) {
  unsigned r;
  asm("v_med3_i32 %0, %1, 0, 1" : "=v"(r) : "v"(v));
  return r;
}
// -v for 8 bf16 (sign bits flipped: exact, 4 v_xor_b32)
__device__ __forceinline__ bf16x8 neg_bf16x8(bf16x8 v) {
  typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
  return __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4_, v) ^ 0x80008000u);
}
// relu-mask bits of a pair of relu'd values (ra, rb >= 0, bit patterns of floats):
// [ra > 0] in bit 0 and [rb > 0] in bit 16 (saturating pack to 16 bits keeps a
// nonzero value nonzero, then a packed min with 1; the inline constant 1 is the low
// half of src1, op_sel_hi:[1,0] reads it for the high half too)
__device__ __forceinline__ unsigned bits01_pair(int ra, int rb) {
  unsigned p, r;
  asm("v_cvt_pk_u16_u32 %0, %1, %2" : "=v"(p) : "v"(ra), "v"(rb));
  asm("v_pk_min_u16 %0, %1, 1 op_sel_hi:[1,0]" : "=v"(r) : "v"(p));
  return r;
}
// the four pair words OR-ed at shifts 0, 2, 4, 6 (element 2d at bit 2d, 2d+1 at bit
// 16+2d) -> the mask byte, element i at bit i (low 8 bits of the result)
__device__ __forceinline__ unsigned pair_bits_to_byte(unsigned q) { return q | (q >> 15); }
// f(integral_constant<int, k>) for k = K .. N-1: compile-time register-array
// indices (a runtime index would put the array in scratch memory)
template <int K, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K < N) {
    f(std::integral_constant<int, K>{});
    static_for<K + 1, N>(f);
  }
}

// (b << e) | acc in one v_lshl_or_b32
template <int E>
__device__ __forceinline__ unsigned lshl_or(unsigned b, unsigned acc) {
  unsigned r;
  asm("v_lshl_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(b), "n"(E), "v"(acc));
  return r;
}
// two fp32 -> packed bf16 pair (RNE, one v_cvt_pk_bf16_f32)
__device__ __forceinline__ unsigned pk_bf16(float a, float b) {
  const bf16x2 v = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(unsigned, v);
}


}  // namespace blk
}  // namespace asr
