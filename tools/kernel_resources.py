"""Per-kernel register / LDS / occupancy summary of one .hip file (hipcc -Rpass-analysis=kernel-resource-usage).

usage: python tools/kernel_resources.py csrc/kernels/<file>.hip [name-filter]
"""
import re
import subprocess
import sys


def main():
    src = __import__("os").path.abspath(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                          "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                         cwd="/tmp").stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        if filt not in n:
            continue
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = n[:n.find("(")] if "(" in n else n
        print(f"{n[:110]:110s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>4} "
              f"spill {r.get('VGPRs Spill', '?'):>3} LDS {r.get('LDS Size [bytes/block]', '?'):>6} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
