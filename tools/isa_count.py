#!/usr/bin/env python3
"""Count gfx950 VALU instructions per SHA-256 compression in this build.

Compiles tiny probe kernels that each run one primitive of
immustore_amd/csrc/sha256_cdna.hpp on per-lane data and counts the vector
ALU instructions in the emitted ISA (minus the probe's own load/store
overhead, measured with an empty probe).  bench.py uses the result to price
the VALU roofline; the output is kept as profiles/isa_counts_rNN.txt.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HDR = os.path.join(ROOT, "immustore_amd", "csrc", "sha256_cdna.hpp")

SRC = r'''
#include "%s"
using namespace mh;
extern "C" __global__ void p_empty(const uint32_t* in, uint32_t* out) {
  int t = blockIdx.x*blockDim.x+threadIdx.x; uint32_t w[16];
  for (int i=0;i<16;i++) w[i]=in[t*16+i];
  for (int i=0;i<8;i++) out[t*8+i]=w[i]^w[i+8];
}
extern "C" __global__ void p_compress(const uint32_t* in, uint32_t* out) {
  int t = blockIdx.x*blockDim.x+threadIdx.x; uint32_t w[16];
  for (int i=0;i<16;i++) w[i]=in[t*16+i];
  State s; s.init(); compress(s,w);
  for (int i=0;i<8;i++) out[t*8+i]=s.h[i]^w[i+8];
}
extern "C" __global__ void p_compress_kw(const uint32_t* in, const uint32_t* kw, uint32_t* out) {
  int t = blockIdx.x*blockDim.x+threadIdx.x; uint32_t w[16];
  for (int i=0;i<16;i++) w[i]=in[t*16+i];
  State s; for (int i=0;i<8;i++) s.h[i]=w[i]; compress_kw(s,kw);
  for (int i=0;i<8;i++) out[t*8+i]=s.h[i]^w[i+8];
}
extern "C" __global__ void p_node(const uint32_t* in, uint32_t* out) {
  int t = blockIdx.x*blockDim.x+threadIdx.x; uint32_t w[16], o[8];
  for (int i=0;i<16;i++) w[i]=in[t*16+i];
  node_hash(w, w+8, o);
  for (int i=0;i<8;i++) out[t*8+i]=o[i];
}
extern "C" __global__ void p_leaf(const uint32_t* in, uint32_t* out) {
  int t = blockIdx.x*blockDim.x+threadIdx.x; uint32_t w[16], o[8];
  for (int i=0;i<16;i++) w[i]=in[t*16+i];
  leaf_hash(w, o);
  for (int i=0;i<8;i++) out[t*8+i]=o[i]^w[i+8];
}
'''


def main():
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.hip")
        open(src, "w").write(SRC % HDR)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-c", src,
                        "-save-temps", "-o", os.path.join(d, "probe.o")], cwd=d, check=True,
                       capture_output=True)
        s = open(os.path.join(d, "probe-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    counts = {}
    for k in ["p_empty", "p_compress", "p_compress_kw", "p_node", "p_leaf"]:
        body = s.split(k + ":")[1].split("s_endpgm")[0]
        ins = [l.split()[0] for l in body.split("\n")
               if l.strip() and not l.strip().startswith((";", ".")) and not l.strip().endswith(":")]
        c = collections.Counter(ins)
        counts[k] = (sum(v for kk, v in c.items() if kk.startswith("v_")), c)
    base = counts["p_empty"][0]
    lines = ["# VALU instructions per primitive, gfx950, hipcc -O3 (probe overhead %d removed)" % base]
    for k in ["p_compress", "p_compress_kw", "p_leaf", "p_node"]:
        v, c = counts[k]
        top = ", ".join("%s %d" % (a, b) for a, b in c.most_common(8) if a.startswith("v_"))
        lines.append("%-14s %5d   (%s)" % (k[2:], v - base, top))
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 1:
        open(sys.argv[1], "w").write(out + "\n")


if __name__ == "__main__":
    main()
