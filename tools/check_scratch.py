"""List every kernel in the built objects whose code object reserves scratch
(private_segment_fixed_size > 0) or spills: extracts each object's gfx950 code
object (.hip_fatbin -> clang-offload-bundler) and reads its AMDGPU metadata
note.  usage: python tools/check_scratch.py [objects...]  (default: csrc/build/*.o)"""
import glob
import os
import re
import subprocess
import sys
import tempfile

BIN = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernels(obj):
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "co.o")
        # an explicit output file: with none, objcopy rewrites the object in
        # place (a newer mtime makes the next make relink for nothing)
        r = subprocess.run([BIN + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, obj,
                            os.path.join(d, "copy.o")], capture_output=True)
        if r.returncode != 0:  # host-only object (no device code)
            return []
        subprocess.run([BIN + "/clang-offload-bundler", "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + fat,
                        "--output=" + co], check=True, capture_output=True)
        notes = subprocess.run([BIN + "/llvm-readelf", "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out, cur = [], {}
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|private_segment_fixed_size|vgpr_count|sgpr_spill_count|"
                     r"vgpr_spill_count):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name" and "name" in cur:
            out.append(cur)
            cur = {}
        cur[k] = v
    if cur:
        out.append(cur)
    return out


def main():
    objs = sys.argv[1:] or sorted(glob.glob(os.path.join(
        ROOT, "calibration-normalizing-flows_amd", "csrc", "build", "*.o")))
    bad = 0
    total = 0
    for o in objs:
        for k in kernels(o):
            if "name" not in k:
                continue
            total += 1
            if int(k.get("private_segment_fixed_size", 0)) > 0:
                bad += 1
                print("%-14s scratch %4s B  vgpr %4s  %s" % (
                    os.path.basename(o), k.get("private_segment_fixed_size"),
                    k.get("vgpr_count"), k["name"][:110]))
    print("%d kernels, %d with scratch" % (total, bad))


if __name__ == "__main__":
    main()
