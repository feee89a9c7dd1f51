"""Build a timing-only variant of libdal.so whose summary_select_kernel (the
fast level 1 of the top-k) stamps s_memrealtime at its phase boundaries into a
device array (dal_k3_trace copies it out; read by scripts/k3_trace.py).  The
product source is not modified: the instrumented copy is compiled from /tmp.
usage: python scripts/k3_trace_build.py OUT_DIR"""
import glob
import os
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
CSRC = os.path.join(REPO, "distributed-active-learning_amd", "csrc")
out = os.path.abspath(sys.argv[1])
os.makedirs(out, exist_ok=True)
s = open(os.path.join(CSRC, "topk.hip")).read()


# K3_TRACE_PATH=rank: the sort stamps 8 / 9 in the rank-selection path (short
# lists) instead of the first match, the region merge; stamp 14 after its
# workspace clear
RANK = os.environ.get("K3_TRACE_PATH") == "rank"
# K3_TRACE_PATH=select: stamps 8 / 9 after the radix pre-selection and after
# the bitonic sort of the long-list path (config 3), slot 15 the compacted count
SELECT = os.environ.get("K3_TRACE_PATH") == "select"
# K3_TRACE_SCORE=1 (with any path): the whole-wave canonical score split in three (max over
# calls, the stamps' waits and atomics included): slot 24 its inputs' loads, 25 the
# divisions, 26 the sequential sum
SCORE = os.environ.get("K3_TRACE_SCORE") == "1"


def sub(old, new, last=False):
    global s
    assert old in s, old[:60]
    if last:
        i = s.rindex(old)
        s = s[:i] + new + s[i + len(old):]
    else:
        s = s.replace(old, new, 1)


sub("struct TopkHdr {", """__device__ unsigned long long g_k3[1024];
#define K3T(slot) do { if (threadIdx.x == 0) g_k3[slot] = __builtin_amdgcn_s_memrealtime(); } while (0)
struct TopkHdr {""")
TAU = next(t for t in ("group_threshold(S, k, stage_issue, stage_rows)", "group_threshold(S, k, prefetch)",
                       "group_threshold(S, k)") if t in s)  # (round 6: the hinted rows' staging runs inside tau)
sub(f"""  const unsigned long long tau = {TAU};
  if (blockIdx.x == 0 && tid == 0) h->kstar = tau;""", f"""  if (blockIdx.x == 0) K3T(0);
  const unsigned long long tau = {TAU};
  if (blockIdx.x == 0) K3T(1);
  if (blockIdx.x == 0 && tid == 0) h->kstar = tau;""")
sub("""  const int nh = static_cast<int>(s_nh);""", """  const int nh = static_cast<int>(s_nh);
  if (blockIdx.x == 0) K3T(2);
  if (tid == 0) g_k3[512 + blockIdx.x] = nh;
  const unsigned long long ta = __builtin_amdgcn_s_memrealtime();""")
sub("""  if (!s_last) return;
  sort_tail_body<true>(AR.ckey, cidx, AR.cpay, h, int64_t{0}, k, out_keys, out_idx, out_scores, tail);
}""", """  K3T(256 + blockIdx.x);
  if (!s_last) return;
  K3T(3);
  if (tid == 0) g_k3[5] = gridDim.x;
  sort_tail_body<true>(AR.ckey, cidx, AR.cpay, h, int64_t{0}, k, out_keys, out_idx, out_scores, tail);
  __syncthreads();
  K3T(6);
}""")
sub("""  if (nv < k) return DAL_KEY_NONE;  // (block-uniform)""", """  if (blockIdx.x == 0) K3T(10);
  if (nv < k) return DAL_KEY_NONE;  // (block-uniform)""")
sub("""  // the upper edge of the k-th key's bucket: >= the k-th group minimum, and at""", """  if (blockIdx.x == 0) K3T(11);
  if (blockIdx.x == 0 && threadIdx.x == 0) g_k3[13] = cnt;
  // the upper edge of the k-th key's bucket: >= the k-th group minimum, and at""")
sub("""  if constexpr (PAY) if (tail.n_reg > 1 && s_runs_sorted &&""", """  if (threadIdx.x == 0) g_k3[4] = m;
  K3T(7);
  if constexpr (PAY) if (tail.n_reg > 1 && s_runs_sorted &&""")
if RANK:
    sub("""      __syncthreads();
    }
    if (tail.clear) {  // every thread read the header above""", """      __syncthreads();
    }
    K3T(8);
    if (tail.clear) {  // every thread read the header above""")
else:
    sub("""      if (PAY) sp[i] = ld_sc1(pay + q);
    }
    __syncthreads();
    if (tail.clear) {  // every thread read the header above""", """      if (PAY) sp[i] = ld_sc1(pay + q);
    }
    __syncthreads();
    K3T(8);
    if (tail.clear) {  // every thread read the header above""")
if RANK:
    sub("""    int tpe = 1;  // lanes per element""", """    __syncthreads();
    K3T(14);
    int tpe = 1;  // lanes per element""")
if SELECT:
    sub("""    loaded = select_compact(keys, idx, pay, M, m, k, sk, si, sp, m);""",
        """    loaded = select_compact(keys, idx, pay, M, m, k, sk, si, sp, m);
  K3T(16);
  if (threadIdx.x == 0) g_k3[15] = m;""")
    sub("""  if (tail.clear) {  // every thread read the header before the first barrier above""",
        """  K3T(17);
  if (tail.clear) {  // every thread read the header before the first barrier above""")
sub("""    if (PAY && h) {
      for (int64_t i = kk + tid; i < k; i += kSortThreads) {""", """    __syncthreads();
    K3T(9);
    if (PAY && h) {
      for (int64_t i = kk + tid; i < k; i += kSortThreads) {""", last=RANK)
sub("""  const int nc = static_cast<int>(s_nc < kept ? s_nc : kept);""", """  const int nc = static_cast<int>(s_nc < kept ? s_nc : kept);
  const unsigned long long tb = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) atomicMax(&g_k3[20], tb - ta);
  if (threadIdx.x == 0) atomicMax(&g_k3[23], static_cast<unsigned long long>(nc));""")
sub("""  // this block's count, then the last block to arrive sorts the candidates""", """  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&g_k3[21], __builtin_amdgcn_s_memrealtime() - tb);""")
sub("""  if (tid == 0) st_sc1(&h->reg_count[blockIdx.x], s_nc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();""", """  if (tid == 0) st_sc1(&h->reg_count[blockIdx.x], s_nc);
  const unsigned long long te = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) atomicMax(&g_k3[22], __builtin_amdgcn_s_memrealtime() - te);""")
s += """
extern "C" int dal_k3_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(dal::g_k3), sizeof(unsigned long long) * 1024) == hipSuccess ? 0 : 1;
}
extern "C" int dal_k3_trace_reset() {
  unsigned long long z[1024] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(dal::g_k3), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
"""
if SCORE:
    sub("""  const uint8_t fl = rerank_flag(R, i);
  const double nr = R.norm64[i];
  const int v = R.votes[i];
  const float* xr = R.x + i * R.ldx;
  double acc = 0.0;
  for (int f0 = 0; f0 < R.d; f0 += 64 * kC) {
    double p[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const int f = f0 + 64 * c + lane;
      p[c] = f < R.d ? (static_cast<double>(xr[f]) / nr) * R.colsum[f] : 0.0;
    }""", """  const unsigned long long t_s = __builtin_amdgcn_s_memrealtime();
  unsigned long long t_l = 0, t_p = 0;
  const uint8_t fl = rerank_flag(R, i);
  const double nr = R.norm64[i];
  const int v = R.votes[i];
  const float* xr = R.x + i * R.ldx;
  double acc = 0.0;
  for (int f0 = 0; f0 < R.d; f0 += 64 * kC) {
    double p[kC];
    float xv[kC];
    double cs[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const int f = f0 + 64 * c + lane;
      xv[c] = f < R.d ? xr[f] : 0.f;
      cs[c] = f < R.d ? R.colsum[f] : 0.0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(xv[0]), "v"(cs[0]), "v"(nr), "v"(v), "v"(static_cast<int>(fl)) : "memory");
    if (f0 == 0) t_l = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      const int f = f0 + 64 * c + lane;
      p[c] = f < R.d ? (static_cast<double>(xv[c]) / nr) * cs[c] : 0.0;
    }
    asm volatile("" ::"v"(p[0]), "v"(p[kC - 1]));
    if (f0 == 0) t_p = __builtin_amdgcn_s_memrealtime();""")
    sub("""  if (!(fl & DAL_ROW_CANDIDATE)) {
    s = __builtin_nan("");
    return false;
  }
  if (fl & DAL_ROW_EXCLUDED) acc = __builtin_nan("");
  // n_lut > 0""", """  asm volatile("" ::"v"(acc));
  if ((threadIdx.x & 63) == 0) {
    const unsigned long long t_c = __builtin_amdgcn_s_memrealtime();
    atomicMax(&g_k3[24], t_l - t_s);
    atomicMax(&g_k3[25], t_p - t_l);
    atomicMax(&g_k3[26], t_c - t_p);
  }
  if (!(fl & DAL_ROW_CANDIDATE)) {
    s = __builtin_nan("");
    return false;
  }
  if (fl & DAL_ROW_EXCLUDED) acc = __builtin_nan("");
  // n_lut > 0""")
# a private directory: a stray common.hpp beside the copy would shadow csrc's
# (the quoted include searches the copy's own directory first)
os.makedirs("/tmp/dal_k3trace", exist_ok=True)
src = "/tmp/dal_k3trace/topk.hip"
open(src, "w").write(s)
hipcc = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
         "-I" + os.path.join(REPO, "include"), "-I" + CSRC]
subprocess.run(hipcc + ["-c", src, "-o", os.path.join(out, "topk.o")], check=True)
objs = [o for o in glob.glob(os.path.join(REPO, "build", "csrc", "*.o")) if not o.endswith("topk.o")]
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                os.path.join(out, "libdal.so")] + objs + [os.path.join(out, "topk.o")], check=True)
print("built", os.path.join(out, "libdal.so"))
