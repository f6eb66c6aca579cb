#!/usr/bin/env python3
"""tools/gen_round_order.py -- diagnostic generator (not product code).

Emits tools/probe_round_order.hip: one wave per SIMD runs the 80 SHA-1 rounds
(message words held in VGPRs, K in an SGPR) written as inline asm in several
instruction orders, and reports cycles per round for each.  Used to find the
order the consumer wave of the pc kernel should issue.
Round i (a=A[i-1], b=A[i-2], c=R[i-3], d=R[i-4], e=R[i-5], R[j]=rotl30(A[j])):
  S: s = add3(e, W, K)        F: f = bitop3(b, c, d)      P: p = rotl5(a)
  T: A[i] = add3(p, f, s)     Q: R[i-2] = rotl30(A[i-2])
"""
import itertools, sys

NA, NR, NT = 8, 8, 4          # ring sizes for A, R and per-round temps
W0, A0, R0 = 0, 16, 24
BASES = {"same": (32, 36, 40), "split": (32, 37, 42), "split2": (33, 38, 43)}


def reg(base, i, n):
    return f"v{base + (i % n)}"


def A(i): return reg(A0, i, NA)
def R(i): return reg(R0, i, NR)


def ops(i, style, bases="same"):
    """instruction dict for round i; style picks how the 5-term sum is formed"""
    P0, F0, S0 = BASES[bases]
    t = i % NT
    p, f, s = f"v{P0 + t}", f"v{F0 + t}", f"v{S0 + t}"
    w = f"v{W0 + (i % 16)}"
    lut = "0xca" if i < 20 else ("0x96" if i < 40 or i >= 60 else "0xe8")
    d = {
        "F": f"v_bitop3_b32 {f}, {A(i - 2)}, {R(i - 3)}, {R(i - 4)} bitop3:{lut}",
        "P": f"v_alignbit_b32 {p}, {A(i - 1)}, {A(i - 1)}, 27",
        "Q": f"v_alignbit_b32 {R(i - 2)}, {A(i - 2)}, {A(i - 2)}, 2",
    }
    if style == "sWK":      # s = e + W + K ; a = p + f + s
        d["S"] = f"v_add3_u32 {s}, {R(i - 5)}, {w}, s20"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
    elif style == "add2":   # S and T as pairs of VOP2 adds
        d["S"] = f"v_add_u32_e32 {s}, {R(i - 5)}, {w}\nv_add_u32_e32 {s}, s20, {s}"
        d["T"] = f"v_add_u32_e32 {A(i)}, {p}, {f}\nv_add_u32_e32 {A(i)}, {A(i)}, {s}"
    elif style == "sadd2":  # S as two VOP2 adds, T as add3
        d["S"] = f"v_add_u32_e32 {s}, {R(i - 5)}, {w}\nv_add_u32_e32 {s}, s20, {s}"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
    elif style == "wk1":    # producer hands over W+K: S is one VOP2 add
        d["S"] = f"v_add_u32_e32 {s}, {R(i - 5)}, {w}"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
    elif style == "wk1b":   # W+K, and e folded into T: T = add3(p, f, e) then + WK
        d["S"] = None
        d["T"] = f"v_add3_u32 {s}, {p}, {f}, {R(i - 5)}\nv_add_u32_e32 {A(i)}, {s}, {w}"
    elif style == "wk3":    # W+K, S = add3(e, WK, f) then T = p + S
        d["S"] = None
        d["T"] = f"v_add3_u32 {s}, {R(i - 5)}, {w}, {f}\nv_add_u32_e32 {A(i)}, {p}, {s}"
    elif style == "vK":     # K in a VGPR instead of an SGPR
        d["S"] = f"v_add3_u32 {s}, {R(i - 5)}, {w}, v47"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
    elif style == "noQ":    # diagnostic: rotl30 replaced by a copy-free xor (wrong math, cost probe)
        d["S"] = f"v_add3_u32 {s}, {R(i - 5)}, {w}, s20"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
        d["Q"] = f"v_xor_b32_e32 {R(i - 2)}, {A(i - 2)}, {A(i - 3)}"
    elif style == "noPQ":   # diagnostic: both rotates replaced by xors
        d["S"] = f"v_add3_u32 {s}, {R(i - 5)}, {w}, s20"
        d["T"] = f"v_add3_u32 {A(i)}, {p}, {f}, {s}"
        d["Q"] = f"v_xor_b32_e32 {R(i - 2)}, {A(i - 2)}, {A(i - 3)}"
        d["P"] = f"v_xor_b32_e32 {p}, {A(i - 1)}, {A(i - 2)}"
    elif style == "sWEF":   # compiler's: s = W + e + f ; a = s + p + K
        d["S"] = None
        d["T"] = None
        d["X"] = f"v_add3_u32 {s}, {w}, {R(i - 5)}, {f}"
        d["T"] = f"v_add3_u32 {A(i)}, {s}, {p}, s20"
    return d


ORDERS = {
    "base/same": ("sWK", "SFPTQ", "", "same"),
    "wk1": ("wk1", "SFPTQ", "", "split"),
    "wk1/lds3": ("wk1", "SFPTQ", "", "split", "lds:3:128:use"),
    "wk1/glb3": ("wk1", "SFPTQ", "", "split", "glb:3:128:use"),
    "wk1/glb3nouse": ("wk1", "SFPTQ", "", "split", "glb:3:128:nouse"),
    "wk1/mix3": ("wk1", "SFPTQ", "", "split", "mix:3:128:use"),
    "wk1/mix3nouse": ("wk1", "SFPTQ", "", "split", "mix:3:128:nouse"),
    "wk1/half3": ("wk1", "SFPTQ", "", "split", "half:3:128:use"),
    "wk1/lds1": ("wk1", "SFPTQ", "", "split", "lds:1:128:use"),
    "wk1/lds3nouse": ("wk1", "SFPTQ", "", "split", "lds:3:128:nouse"),
    "wk1/lds3b64": ("wk1", "SFPTQ", "", "split", "lds:3:64:use"),
    "base/lds3": ("sWK", "SFPTQ", "", "split", "lds:3:128:use"),
    "wk1/PQFST": ("wk1", "PQFST", "", "split"),
    "wk1b": ("wk1b", "FPTQ", "", "split"),
    "wk3": ("wk3", "FPTQ", "", "split"),
    "wk3/QFPT": ("wk3", "QFPT", "", "split"),
    "vK": ("vK", "SFPTQ", "", "split"),
    "base/split": ("sWK", "SFPTQ", "", "split"),
    "base/split2": ("sWK", "SFPTQ", "", "split2"),
    "add2/split": ("add2", "SFPTQ", "", "split"),
    "sadd2/split": ("sadd2", "SFPTQ", "", "split"),
    "noQ/split": ("noQ", "SFPTQ", "", "split"),
    "noPQ/split": ("noPQ", "SFPTQ", "", "split"),
}
_OLD_ORDERS = {
    # name: (style, per-round order, lookahead: ops of round i+1 issued at the end of round i)
    "SFPTQ": ("sWK", "SFPTQ", ""),
    "PSFTQ": ("sWK", "PSFTQ", ""),
    "QPSFT": ("sWK", "QPSFT", ""),
    "PQSFT": ("sWK", "PQSFT", ""),
    "SFQPT": ("sWK", "SFQPT", ""),
    "PSQFT": ("sWK", "PSQFT", ""),
    "PTQ+SF": ("sWK", "PTQ", "SF"),      # S,F of the next round hoisted before its P
    "PTQ+S": ("sWK", "PFTQ", "S"),
    "FXPTQ": ("sWEF", "FXPTQ", ""),
    "FPXTQ": ("sWEF", "FPXTQ", ""),
    "PFXQT": ("sWEF", "PFXQT", ""),
}


def lds_feed(name):
    spec = ORDERS[name][4] if len(ORDERS[name]) > 4 else ""
    if not spec:
        return None
    src, depth, width, use = spec.split(":")
    return int(depth), int(width), use == "use", src


def body(name):
    style, order, ahead, bases = ORDERS[name][:4]
    feed = lds_feed(name)
    out = []
    issued = set()
    if feed:
        depth, width, use, src = feed
        dst = (lambda q: f"v[{4 * (q % 4)}:{4 * (q % 4) + 3}]") if use else (lambda q: "v[48:51]")

        def rd(q):
            if src == "glb":     # L2-resident global buffer, [20][64] uint4
                return [f"global_load_dwordx4 {dst(q)}, %2, off offset:{q * 1024 - 2048 if q * 1024 >= 2048 else q * 1024}"] \
                    if False else [f"global_load_dwordx4 {dst(q)}, %2, off offset:{(q % 4) * 1024}"]
            if src == "mix" and q % 2 == 1:
                return [f"global_load_dwordx4 {dst(q)}, %2, off offset:{(q % 4) * 1024}"]
            if src == "half":    # ds_read with only 32 lanes enabled
                return ["s_mov_b32 s21, exec_hi", "s_mov_b32 exec_hi, 0",
                        f"ds_read_b128 {dst(q)}, %1 offset:{q * 1024}", "s_mov_b32 exec_hi, s21"]
            if width == 128:
                return [f"ds_read_b128 {dst(q)}, %1 offset:{q * 1024}"]
            r = dst(q).strip("v[]").split(":")
            lo = int(r[0])
            return [f"ds_read_b64 v[{lo}:{lo + 1}], %1 offset:{q * 1024}",
                    f"ds_read_b64 v[{lo + 2}:{lo + 3}], %1 offset:{q * 1024 + 8}"]
        per = 1 if width == 128 else 2
        for q in range(min(depth, 20)):
            out += rd(q)
    for i in range(80):
        if feed and i % 4 == 0:
            q = i // 4
            if q + depth < 20:
                out += rd(q + depth)
            after = min(depth, 19 - q) * per   # reads issued after quad q's
            if src == "glb":
                out.append(f"s_waitcnt vmcnt({after})")
            elif src in ("mix", "mix3b"):
                # same-type reads issued after quad q's: odd quads go to VMEM
                later = [r for r in range(q + 1, min(q + depth, 19) + 1)]
                same = sum(1 for r in later if (r % 2) == (q % 2))
                out.append(f"s_waitcnt vmcnt({same})" if q % 2 == 1 else f"s_waitcnt lgkmcnt({same})")
            else:
                out.append(f"s_waitcnt lgkmcnt({after})")
        d = ops(i, style, bases)
        for c in order:
            if (i, c) not in issued:
                out.extend(d[c].split("\n")); issued.add((i, c))
        if ahead and i + 1 < 80:
            d1 = ops(i + 1, style, bases)
            for c in ahead:
                out.extend(d1[c].split("\n")); issued.add((i + 1, c))
    return out


def main():
    lines = ['// GENERATED by tools/gen_round_order.py -- diagnostic probe, not product code',
             '#include <hip/hip_runtime.h>', '#include <stdio.h>']
    clob = ", ".join(f'"v{r}"' for r in range(0, 52)) + ', "s20"'
    names = list(ORDERS)
    for k, name in enumerate(names):
        asm = "\\n".join(body(name))
        lines += [f'__global__ void __launch_bounds__(64) k{k}(int iters, unsigned long long* clk, unsigned* out) {{',
                  '  __shared__ uint4 lbuf[20 * 64];',
                  '  for (int q = 0; q < 20; ++q) lbuf[q * 64 + threadIdx.x] = make_uint4(q, threadIdx.x, 1, 2);',
                  '  __syncthreads();',
                  '  unsigned laddr = (unsigned)(uintptr_t)(lbuf + threadIdx.x);',
                  '  const uint4* gaddr = reinterpret_cast<const uint4*>(out) + 4096 + threadIdx.x;',
                  '  unsigned x = threadIdx.x;',
                  '  unsigned long long t0 = __builtin_amdgcn_s_memtime();',
                  '  asm volatile("s_mov_b32 s20, 0x5a827999" ::: "s20");',
                  '  for (int it = 0; it < iters; ++it) {',
                  f'    asm volatile("{asm}" : "+v"(x) : "v"(laddr), "v"(gaddr) : {clob}, "s21", "memory");',
                  '  }',
                  '  unsigned long long t1 = __builtin_amdgcn_s_memtime();',
                  '  out[blockIdx.x * 64 + threadIdx.x] = x;',
                  '  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;',
                  '}']
    lines.append('template <typename K> static double run(K k, int blocks) {')
    lines.append('  unsigned long long* clk; unsigned* out; hipMalloc(&clk, blocks * 8); hipMalloc(&out, blocks * 256 + (4096 + 4 * 64) * 16); hipMemset(out, 0, blocks * 256 + (4096 + 4 * 64) * 16);')
    lines.append('  const int iters = 64;')
    lines.append('  for (int r = 0; r < 2; ++r) { hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, iters, clk, out); hipDeviceSynchronize(); }')
    lines.append('  unsigned long long h[1024]; hipMemcpy(h, clk, blocks * 8, hipMemcpyDeviceToHost);')
    lines.append('  double c = 0; for (int b = 0; b < blocks; ++b) c += h[b]; hipFree(clk); hipFree(out);')
    lines.append('  return c / blocks / (iters * 80.0);')
    lines.append('}')
    lines.append('int main() {')
    lines.append('  printf("%-8s %12s %12s\\n", "order", "cyc/round", "cyc/instr");')
    for k, name in enumerate(names):
        n = sum(1 for x in body(name) if x.startswith("v_")) / 80.0
        lines.append(f'  {{ double c = run(k{k}, 256); printf("%-8s %12.2f %12.2f\\n", "{name}", c, c / {n}); }}')
    lines.append('  return 0;\n}')
    open(sys.argv[1] if len(sys.argv) > 1 else "tools/probe_round_order.hip", "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
