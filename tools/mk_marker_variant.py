"""Debug aid: a copy of the library whose device-plan kernels record, from block 0, a start marker
(sequence number << 8 | kernel code) into host-mapped memory, readable after a GPU fault through
mm_debug_marks.  Writes ab_variants/marks/csrc; build with tools/build_variant.sh conventions."""
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = os.path.join(ROOT, "ab_variants", "marks")
shutil.rmtree(d, ignore_errors=True)
os.makedirs(os.path.join(d, "csrc"))
os.makedirs(os.path.join(d, "include"))
src = os.path.join(ROOT, "vvc-extension-mm_amd", "csrc")
for f in os.listdir(src):
    shutil.copy(os.path.join(src, f), os.path.join(d, "csrc", f))
shutil.copy(os.path.join(ROOT, "include", "mm360.h"), os.path.join(d, "include"))
for f in os.listdir(os.path.join(d, "csrc")):
    p = os.path.join(d, "csrc", f)
    s = open(p).read().replace('"../../include/mm360.h"', '"../include/mm360.h"')
    open(p, "w").write(s)
p = os.path.join(d, "csrc", "mm_kernels.hip")
s = open(p).read()
hdr = '''
__device__ unsigned int* g_mark;
__device__ unsigned int g_mark_seq;
#define MM_MARK(code)                                                                   \\
  do {                                                                                  \\
    if (g_mark && blockIdx.x == 0 && threadIdx.x == 0) {                                \\
      const unsigned s_ = atomicAdd(&g_mark_seq, 1u);                                   \\
      __hip_atomic_store(&g_mark[s_ & 63], (s_ << 8) | (code), __ATOMIC_RELAXED,        \\
                         __HIP_MEMORY_SCOPE_SYSTEM);                                    \\
    }                                                                                   \\
  } while (0)
'''
s = s.replace("namespace {\n", "namespace {\n" + hdr, 1)
codes = {"k_plan_count": 1, "k_plan_place": 2, "k_dmvr_setup_dev": 3, "k_dmvr_reproj_dev": 4,
         "k_dmvr_search_dev": 5, "k_setup_dev": 6, "k_reproj_dev": 7, "k_mc_dev": 8}
for k, code in codes.items():
    m = re.search(r"__global__[^{;]*\b" + k + r"\(", s)
    assert m, k
    brace = s.index("{", m.end())
    # the parameter list may hold no braces; insert after the opening brace of the body
    s = s[:brace + 1] + f"\n  MM_MARK({code});" + s[brace + 1:]
host = '''
static unsigned int* h_mark_host = nullptr;
extern "C" int mm_debug_marks(unsigned int* out) {
  if (!h_mark_host) return -1;
  for (int i = 0; i < 64; i++) out[i] = reinterpret_cast<volatile unsigned int*>(h_mark_host)[i];
  return 0;
}
static void mark_init() {
  if (h_mark_host) return;
  if (hipHostMalloc(reinterpret_cast<void**>(&h_mark_host), 64 * sizeof(unsigned int),
                    hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return;
  for (int i = 0; i < 64; i++) h_mark_host[i] = 0;
  unsigned int* dp = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&dp), h_mark_host, 0) != hipSuccess) return;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_mark), &dp, sizeof(dp));
}
'''
i = s.index("int mm_create(const mm_seq_params* p, int device, mm_ctx** out_ctx) {")
s = s[:i] + host + s[i:]
j = s.index("{", i + len(host)) + 1
s = s[:j] + "\n  mark_init();" + s[j:]
open(p, "w").write(s)
print("wrote", d)
