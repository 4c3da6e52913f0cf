"""Regenerate tools/rs_stamps.patch (the resample's phase clocks, a timing-only
variant) from the current product sources: the clock hooks are inserted at
stable anchors of k_resample1 and the diff against the sources is written.

python tools/regen_rs_stamps.py      (then: python tools/variants.py build rs_stamps)
"""
import difflib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gen_amd", "csrc")

MACROS = '''// timing-only variants (results wrong): GH_RS_EXIT=k leaves k_resample1 after
// phase k (0 start, 1 fold, 2 quantise + scan, 3 grid barrier), to price the
// phases including the launch
#if defined(GH_RS_EXIT)
#define GH_RS_EXIT_AT(k) \\
  if (GH_RS_EXIT == (k)) return;
#else
#define GH_RS_EXIT_AT(k)
#endif

#if defined(GH_RS_STAMPS)  // timing-only variant: per-block phase clocks
static __device__ uint64_t g_rs_stamps[1024 * 16];
#define GH_RS_STAMP(k) \\
  if (threadIdx.x == 0 && blockIdx.x < 1024) g_rs_stamps[blockIdx.x * 16 + (k)] = wall_clock64();
// per wave of the marks phase: [clock before the first slot count, clock
// after the loop, wave-wide carry loops | exact slot counts << 32, carries those wrote]
static __device__ uint64_t g_rs_wave[1024 * 16 * 4];
// where the block runs: the HW_ID register (wave, SIMD, CU, SH, SE ids) and the XCC id
#define GH_RS_PLACE() \\
  if (threadIdx.x == 0 && blockIdx.x < 1024) { \\
    g_rs_stamps[blockIdx.x * 16 + 8] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4); \\
    g_rs_stamps[blockIdx.x * 16 + 9] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 20); \\
  }
#else
#define GH_RS_STAMP(k)
#define GH_RS_PLACE()
#endif

'''

API = '''#if defined(GH_RS_STAMPS)
extern "C" int gh_debug_rs_stamps(uint64_t* out, int n) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rs_stamps), sizeof(uint64_t) * (size_t)n));
  return GH_OK;
}
extern "C" int gh_debug_rs_waves(uint64_t* out, int n) {
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rs_wave), sizeof(uint64_t) * (size_t)n));
  return GH_OK;
}
#endif

'''


def insert(s, lo, anchor, text, after=True):
    """insert text after (or before) the first occurrence of anchor at or past lo"""
    i = s.index(anchor, lo)
    j = i + len(anchor) if after else i
    return s[:j] + text + s[j:]


def stamped_kernels(s):
    head = "template <bool MARKS, int IT, bool SUMS>\n__global__ __launch_bounds__(kRsBlock"
    s = insert(s, 0, head, MACROS, after=False)
    k0 = s.index(head)
    end = s.index("// ------------------------------------------------ multi-rank resample", k0)
    body = s[k0:end]
    b = body
    b = insert(b, 0, "__shared__ int sfail;  // the barrier wait timed out: write nothing\n",
               "  GH_RS_STAMP(0);\n  GH_RS_PLACE();\n  GH_RS_EXIT_AT(0);\n")
    b = insert(b, 0, "M = amax_value(readlane63_u64(key));\n", "    GH_RS_STAMP(7);\n")
    b = insert(b, 0, "M = blk16_max1(m, smd);\n", "    GH_RS_STAMP(7);\n    GH_RS_EXIT_AT(1);\n")
    b = insert(b, 0, "  auto commit = [&]() {", "  GH_RS_STAMP(1);\n", after=False)
    b = insert(b, 0, "blk16_scan<false>(tsum, &s1, &s2, smu, smd);\n", "  GH_RS_STAMP(2);\n  GH_RS_EXIT_AT(2);\n")
    b = insert(b, 0, "  if (threadIdx.x == 0) {\n    uint64_t all = 0, before = 0;", "  GH_RS_STAMP(3);\n",
               after=False)
    b = insert(b, b.index("GH_RS_STAMP(3)"), "  if (sfail) return;\n", "  GH_RS_EXIT_AT(3);\n  GH_RS_STAMP(4);\n")
    b = insert(b, 0, "const uint32_t N = (uint32_t)r.mk.n_global;  // < 2^31: 32-bit slots and groups\n",
               "#if defined(GH_RS_STAMPS)\n  const uint64_t wt0 = wall_clock64();\n  uint64_t wmany = 0, wcar = 0, wnear = 0;\n#endif\n")
    b = insert(b, 0, "    if (near) j = sys_count_exact_call(&sd, N, X);",
               "#if defined(GH_RS_STAMPS)\n    wnear += __builtin_popcountll(__builtin_amdgcn_ballot_w64(near));\n#endif\n",
               after=False)
    b = insert(b, 0, "uint64_t bm = __builtin_amdgcn_ballot_w64(many);\n",
               "#if defined(GH_RS_STAMPS)\n    wmany += __builtin_popcountll(bm);\n#endif\n")
    b = insert(b, 0, "a1 = __builtin_amdgcn_readlane((int32_t)g1, L);\n",
               "#if defined(GH_RS_STAMPS)\n      wcar += (uint64_t)(a1 - a0);\n#endif\n")
    loop_end = "    s_i = e_i;\n  }\n"
    i = b.rindex(loop_end) + len(loop_end)
    b = b[:i] + '''#if defined(GH_RS_STAMPS)
  if ((threadIdx.x & 63) == 0 && blockIdx.x < 1024) {
    uint64_t* wp = g_rs_wave + ((uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6)) * 4;
    wp[0] = wt0;
    wp[1] = wall_clock64();
    wp[2] = wmany | (wnear << 32);
    wp[3] = wcar;
  }
#endif
  GH_RS_STAMP(5);
''' + b[i:]
    j = b.rstrip("\n").rindex("\n}")  # the kernel's closing brace
    b = b[:j] + "\n  GH_RS_STAMP(6);" + b[j:]
    return s[:k0] + b + s[end:]


def main():
    out = []
    for name, fn in (("gh_kernels.h", stamped_kernels),
                     ("gh_api.hip", lambda s: insert(s, 0, "// ------------------------------------------------------------------ PMMH",
                                                     API, after=False))):
        src = open(os.path.join(CSRC, name)).read()
        new = fn(src)
        out += difflib.unified_diff(src.splitlines(True), new.splitlines(True), f"a/{name}", f"b/{name}")
    open(os.path.join(ROOT, "tools", "rs_stamps.patch"), "w").write("".join(out))
    print("wrote tools/rs_stamps.patch")


if __name__ == "__main__":
    main()
