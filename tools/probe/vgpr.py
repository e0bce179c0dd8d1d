"""Compile b3_kernels.hip with source edits (compile-only probes) and print leaf VGPRs."""
import subprocess, sys
SRC = "/root/repo/syncr_amd/csrc/b3_kernels.hip"
def probe(edits):
    s = open(SRC).read()
    for a, b in edits:
        assert a in s, a[:60]
        s = s.replace(a, b)
    open("/tmp/exp.hip", "w").write(s)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "/tmp/exp.hip",
                        "-o", "/tmp/exp.o", "-I", "/root/repo/include", "-I", "/root/repo/syncr_amd/csrc",
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
    out, on = [], False
    for l in r.stderr.splitlines():
        if "Function Name" in l: on = "b3_leaf_kernelILb0ELi0" in l
        if on and ("VGPRs:" in l or "Scratch" in l or "Occupancy" in l): out.append(l.split("remark:")[1].strip())
    return out or r.stderr[-2000:]
VARIANTS = {
    "cur": [],
    "root_uniform": [("            root = !tail;", "            root = true;")],
    "no_tail_path": [("                tail = (code & B3_TAIL) != 0;", "                tail = false;")],
    "no_placeholder_skip": [("            if (code & B3_TAIL) continue;                        // placeholder: hashed as a packed unit\n", "")],
}
for n in (sys.argv[1:] or VARIANTS):
    print(n, probe(VARIANTS[n]), flush=True)
