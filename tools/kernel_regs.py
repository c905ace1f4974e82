"""VGPR / AGPR / scratch / LDS of the scan kernels in built libraries.

    python tools/kernel_regs.py scann_amd/lib/libscann_mi355x.so [more.so ...] [--match lut16_scan]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(lib):
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib])
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fb}",
                               f"--output={co}"])
        notes = subprocess.check_output([f"{LLVM}/llvm-readelf", "--notes", co], text=True)
    for e in notes.split("  - .agpr_count")[1:]:
        f = lambda k: (re.search(rf"\.{k}:\s+(\S+)", e) or [None, None])[1]
        yield dict(name=f("name"), vgpr=f("vgpr_count"), agpr=e.split()[1],
                   scratch=f("private_segment_fixed_size"), lds=f("group_segment_fixed_size"))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    pat = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "lut16_scan"
    args = [a for a in args if a != pat]
    for lib in args:
        for k in kernels(lib):
            if re.search(pat, k["name"] or ""):
                print(f"{os.path.basename(lib):32s} {k['name'][:70]:70s} vgpr={k['vgpr']} "
                      f"agpr={k['agpr']} scratch={k['scratch']} lds={k['lds']}")
