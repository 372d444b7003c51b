"""Engine shares of a per-step kernel table (scripts/rocpd_steps.py output).

    python scripts/kernel_shares.py gpurun_out/rn5_steps.txt [more.txt ...]

Groups every kernel line (`us/step calls/step avg_us pct name`) by engine:
hipBLASLt (`Cijk_*`), MIOpen / CK convolutions, the in-tree GEMM
(`dtfk::gemm2::`), the in-tree 3x3 convolution (`dtfk::cig::`), in-tree
BatchNorm (`dtfk::bn::`), other in-tree kernels (`dtfk::`), and the rest
(torch elementwise / MIOpen glue / fills).
"""
import re
import sys

GROUPS = [
    ("hipBLASLt", lambda k: k.startswith("Cijk_")),
    ("MIOpen/CK conv", lambda k: "dtfk::" not in k and (
        k.startswith(("igemm_", "naive_conv", "MIOpen")) or "ck::" in k or k.startswith("_ZN2ck")
        or "conv_fwd" in k or "conv_bwd" in k or "gridwise_convolution" in k)),
    ("in-tree gemm_big", lambda k: "dtfk::gemm2::" in k),
    ("in-tree conv (implicit GEMM)", lambda k: "dtfk::cig::" in k),
    ("in-tree BN", lambda k: "dtfk::bn::" in k),
    ("other in-tree", lambda k: "dtfk::" in k),
    ("other (torch / MIOpen glue)", lambda k: True),
]


def main():
    for path in sys.argv[1:]:
        total, per = None, {g: 0.0 for g, _ in GROUPS}
        for line in open(path):
            m = re.match(r"window .* per step ([0-9.]+) us", line.strip())
            if m:
                total = float(m.group(1))
                continue
            m = re.match(r"\s*([0-9.]+)\s+([0-9.]+)\s+([0-9.]+)\s+([0-9.]+)\s+(.*)$", line)
            if not m:
                continue
            us, name = float(m.group(1)), m.group(5).strip()
            for g, pred in GROUPS:
                if pred(name):
                    per[g] += us
                    break
        tot = total or sum(per.values())
        print(f"{path}: per step {tot:.1f} us")
        for g, _ in GROUPS:
            if per[g]:
                print(f"  {g:<30} {per[g]:9.1f} us  {100 * per[g] / tot:5.1f} %")


if __name__ == "__main__":
    main()
