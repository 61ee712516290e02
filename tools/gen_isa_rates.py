"""Generate tools/isa_rates.hip: per-instruction issue cost on gfx950 for the
integer instruction mix of Goldilocks arithmetic (Poseidon, NTT, quotient).

Each kernel runs one instruction in 8 independent chains per lane for ITERS
iterations between two s_memtime reads (shader-clock ticks, MI355X_MICROARCH.md
"s_memtime tick = shader cycle"), so the result is in cycles and needs no clock
assumption.  Dispatches last tens of milliseconds (launch ramp negligible) and
run at 1, 4 and 8 waves per SIMD; the per-SIMD issue cost of an instruction is
cycles / (waves per SIMD x instructions per wave).

    python tools/gen_isa_rates.py > tools/isa_rates.hip
    hipcc --offload-arch=gfx950 -O3 tools/isa_rates.hip -o tools/isa_rates && tools/isa_rates
"""
import sys

# name, asm template over %0 (u32 dst/src chain), %1 (u32 other), 64-bit chains use w
# (kind: 32 = chain in u[], 64 = chain in w[] (64-bit VGPR pair))
INSTRS = [
    ("v_add_u32", 32, "v_add_u32_e32 %0, %0, %1"),
    ("v_xor_b32", 32, "v_xor_b32_e32 %0, %1, %0"),
    ("v_add3_u32", 32, "v_add3_u32 %0, %0, %1, %0"),
    ("v_add_co_u32_e64", 32, "v_add_co_u32_e64 %0, s[40:41], %0, %1"),
    ("v_addc_co_u32_e64", 32, "v_addc_co_u32_e64 %0, s[42:43], %0, %1, s[40:41]"),
    ("v_cndmask_b32_e64", 32, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]"),
    ("v_mul_lo_u32", 32, "v_mul_lo_u32 %0, %0, %1"),
    ("v_mul_hi_u32", 32, "v_mul_hi_u32 %0, %0, %1"),
    ("v_mul_u32_u24", 32, "v_mul_u32_u24_e32 %0, 13, %0"),
    ("v_mad_u32_u24", 32, "v_mad_u32_u24 %0, %0, 13, %1"),
    ("v_mul_hi_u32_u24", 32, "v_mul_hi_u32_u24_e32 %0, 13, %0"),
    ("v_mul_u32_u24_vv", 32, "v_mul_u32_u24_e32 %0, %1, %0"),
    ("v_alignbit_b32", 32, "v_alignbit_b32 %0, %0, %1, 7"),
    ("v_lshlrev_b32", 32, "v_lshlrev_b32_e32 %0, 3, %0"),
    ("v_mad_u64_u32", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0"),
    ("v_mad_u64_u32_vv", 64, "v_mad_u64_u32 %0, s[40:41], %1, %1, %0"),
    ("v_lshl_add_u64", 64, "v_lshl_add_u64 %0, %0, 0, %2"),
    ("v_lshlrev_b64", 64, "v_lshlrev_b64 %0, 3, %0"),
    ("v_mov_b64", 64, "v_mov_b64 %0, %2"),
    ("v_fma_f32", 0, "v_fma_f32 %0, %0, %1, %1"),
    # VOP2 carry forms through VCC (the e32 encodings of the ops above)
    ("v_add_co_u32_e32", 32, "v_add_co_u32_e32 %0, vcc, %0, %1"),
    ("v_addc_co_u32_e32", 32, "v_addc_co_u32_e32 %0, vcc, %0, %1, vcc"),
    ("v_subb_co_u32_e32", 32, "v_subb_co_u32_e32 %0, vcc, %0, %1, vcc"),
    ("v_cndmask_b32_e32", 32, "v_cndmask_b32_e32 %0, %0, %1, vcc"),
    ("v_mad_u64_u32_vcc", 64, "v_mad_u64_u32 %0, vcc, %1, 13, %0"),
]
# hazard-pad cost: VALU instructions with the wait states the gfx950 hazard
# rules make hipcc insert, per VALU instruction (4th field = VALU count)
NOPS = [
    ("mad", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1),
    ("mad+s_nop0", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0\\n\\ts_nop 0", 1),
    ("mad+2xs_nop0", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0\\n\\ts_nop 0\\n\\ts_nop 0", 1),
    ("mad+s_nop1", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0\\n\\ts_nop 1", 1),
    ("addco,addc", 32, "v_add_co_u32_e64 %0, s[40:41], %0, %1\\n\\tv_addc_co_u32_e64 %0, s[42:43], %0, %1, s[40:41]", 2),
    ("addco,addc e32", 32, "v_add_co_u32_e32 %0, vcc, %0, %1\\n\\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc", 2),
    ("addco e32,cndmask e32", 32, "v_add_co_u32_e32 %0, vcc, %0, %1\\n\\tv_cndmask_b32_e32 %0, %0, %1, vcc", 2),
    ("addco,2nop,addc", 32, "v_add_co_u32_e64 %0, s[40:41], %0, %1\\n\\ts_nop 0\\n\\ts_nop 0\\n\\tv_addc_co_u32_e64 %0, s[42:43], %0, %1, s[40:41]", 2),
]
# dependency distance: the 8 statements per iteration cycle over CH chains,
# so each instruction depends on the one CH statements earlier (CH = 8: the
# throughput tables above; CH = 1: a single dependent chain per wave)
CHAINS = [
    ("mad CH1", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1, 1),
    ("mad CH2", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1, 2),
    ("mad CH4", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1, 4),
    ("mad CH8", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1, 8),
    ("add_u32 CH1", 32, "v_add_u32_e32 %0, %0, %1", 1, 1),
    ("add_u32 CH2", 32, "v_add_u32_e32 %0, %0, %1", 1, 2),
    ("cndmask CH1", 32, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]", 1, 1),
    ("cndmask CH2", 32, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]", 1, 2),
]
# one asm statement holding the 8 chains' instructions (no compiler hazard pad
# between them: inline asm that writes an SGPR gets an s_nop after it); the
# clean per-class costs for tools/issue_ceiling.py
BLOCKS = [
    ("mad blk", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0", 1, -1),
    ("mad+nop blk", 64, "v_mad_u64_u32 %0, s[40:41], %1, 13, %0\\n\\ts_nop 0", 1, -1),
    ("add_u32 blk", 32, "v_add_u32_e32 %0, %0, %1", 1, -1),
    ("mov_b32 blk", 32, "v_mov_b32_e32 %0, %1", 1, -1),
    ("cndmask blk", 32, "v_cndmask_b32_e64 %0, %0, %1, s[40:41]", 1, -1),
    ("sub_co blk", 32, "v_sub_co_u32_e64 %0, s[42:43], %0, %1", 1, -1),
    ("mul_u24 blk", 32, "v_mul_u32_u24_e32 %0, %1, %0", 1, -1),
    ("mul_hi_u24 blk", 32, "v_mul_hi_u32_u24_e32 %0, %1, %0", 1, -1),
    ("mad_u32_u24 blk", 32, "v_mad_u32_u24 %0, %0, %1, %0", 1, -1),
]
ITERS = 65536


def kernel(i, name, kind, asm, nvalu=1, ch=8):
    lines = []
    if kind == 64:
        decl = "uint64_t c[8]; for (int i = 0; i < 8; i++) c[i] = seed + i + threadIdx.x;"
        cons = '"+v"(c[{k}]) : "v"(x), "v"(z) : "s40","s41","s42","s43","vcc"'
    elif kind == 0:
        decl = "float c[8]; for (int i = 0; i < 8; i++) c[i] = 1.0f + i * 1e-3f;"
        cons = '"+v"(c[{k}]) : "v"(g) : "s40","s41","s42","s43","vcc"'
    else:
        decl = "uint32_t c[8]; for (int i = 0; i < 8; i++) c[i] = seed + i + threadIdx.x;"
        cons = '"+v"(c[{k}]) : "v"(x) : "s40","s41","s42","s43","vcc"'
    if ch < 0:  # block: chains %0..%7, x = %8, z = %9
        ins = "\\n\\t".join(asm.replace("%1", "%8").replace("%2", "%9").replace("%0", f"%{k}") for k in range(8))
        outs = ", ".join(f'"+v"(c[{k}])' for k in range(8))
        ins_c = '"v"(x), "v"(z)' if kind != 0 else '"v"(g), "v"(g)'
        body = f'    asm volatile("{ins}" : {outs} : {ins_c} : "s40","s41","s42","s43","vcc");'
    else:
        body = "\n".join(f'    asm volatile("{asm}" : {cons.format(k=k % ch)});' for k in range(8))
    lines.append(f"""__global__ void k{i}(uint64_t *out, uint64_t *ticks, uint32_t seed) {{
  // {name}
  {decl}
  uint32_t x = seed * 3 + threadIdx.x; uint64_t z = seed * 7ull + threadIdx.x; float g = 1.0001f;
  (void)x; (void)z; (void)g;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < ITERS; it++) {{
{body}
  }}
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint64_t s = 0;
  for (int i = 0; i < 8; i++) s += (uint64_t)c[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) ticks[(blockIdx.x * blockDim.x + threadIdx.x) / 64] = t1 - t0;
}}""")
    return "\n".join(lines)


def main():
    global INSTRS
    if len(sys.argv) > 1 and sys.argv[1] == "nops":
        INSTRS = NOPS
    elif len(sys.argv) > 1 and sys.argv[1] == "all":
        INSTRS = INSTRS + NOPS
    elif len(sys.argv) > 1 and sys.argv[1] == "chains":
        INSTRS = CHAINS + BLOCKS
    INSTRS = [t if len(t) >= 4 else t + (1,) for t in INSTRS]
    INSTRS = [t if len(t) == 5 else t + (8,) for t in INSTRS]
    print("// isa_rates.hip -- GENERATED by tools/gen_isa_rates.py; see that file.")
    print("#include <hip/hip_runtime.h>\n#include <stdint.h>\n#include <stdio.h>\n#include <vector>")
    print(f"#define ITERS {ITERS}")
    for i, (name, kind, asm, nv, ch) in enumerate(INSTRS):
        print(kernel(i, name, kind, asm, nv, ch))
    nvs = ", ".join(str(t[3]) for t in INSTRS)
    names = ", ".join(f'"{t[0]}"' for t in INSTRS)
    ptrs = ", ".join(f"k{i}" for i in range(len(INSTRS)))
    print(f"""
typedef void (*KFn)(uint64_t *, uint64_t *, uint32_t);
int main() {{
  const char *names[] = {{{names}}};
  const int nvalu[] = {{{nvs}}};
  KFn fns[] = {{{ptrs}}};
  int cus = 256;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, 0) == hipSuccess) cus = p.multiProcessorCount;
  const int wps_list[] = {{1, 4, 8}};
  uint64_t *out, *ticks;
  hipMalloc(&out, (size_t)cus * 4 * 8 * 64 * 8);
  hipMalloc(&ticks, (size_t)cus * 4 * 8 * 8);
  printf("%-20s %s\\n", "instruction", "cycles per wave-instruction per SIMD at 1 / 4 / 8 waves per SIMD (s_memtime)");
  for (int k = 0; k < {len(INSTRS)}; k++) {{
    printf("%-20s", names[k]);
    for (int wps : wps_list) {{
      // cus * wps workgroups of 4 waves (one per SIMD): wps waves per SIMD
      const int nw = cus * 4 * wps;
      fns[k]<<<cus * wps, 256>>>(out, ticks, 1);
      hipDeviceSynchronize();
      hipEvent_t a, b;
      hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      fns[k]<<<cus * wps, 256>>>(out, ticks, 2);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0; hipEventElapsedTime(&ms, a, b);
      std::vector<uint64_t> t(nw);
      hipMemcpy(t.data(), ticks, nw * 8, hipMemcpyDeviceToHost);
      double avg = 0; for (auto v : t) avg += (double)v; avg /= nw;
      printf("  %6.2f (%5.1f ms)", avg / (8.0 * ITERS * nvalu[k]) / wps, ms);
    }}
    printf("\\n");
  }}
  return 0;
}}""")


if __name__ == "__main__":
    main()
