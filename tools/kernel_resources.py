"""Per-kernel resource metadata of the built library (CPU only, no GPU): every
gfx950 code object embedded in opencv_amd/lib/libtbdk.so (the clang offload
bundles hipcc -shared writes, one per translation unit) is cut out by its ELF
header and read with llvm-readelf --notes; the AMDGPU metadata gives, per
kernel, its static LDS (.group_segment_fixed_size), scratch
(.private_segment_fixed_size), VGPR / SGPR counts and spills.

  python tools/kernel_resources.py [lib.so]      # table of every kernel

tests/test_kernel_resources.py uses it to hold the hot kernels to their
intended resources (no scratch anywhere, no LDS in the streaming pyramid
kernels: a runtime-indexed private array that the compiler moves to LDS
serialized the two-role pyramid's loads, +10 us per 1080p build).
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
FIELDS = (".group_segment_fixed_size", ".private_segment_fixed_size", ".vgpr_count", ".sgpr_count",
          ".vgpr_spill_count", ".sgpr_spill_count")


def code_objects(data: bytes):
    """device ELF images inside a host shared object (every ELF but the host's own)"""
    out = []
    pos = data.find(b"\x7fELF", 1)
    while pos > 0:
        hdr = data[pos:pos + 64]
        if len(hdr) == 64 and hdr[4] == 2 and hdr[5] == 1:  # ELFCLASS64, little endian
            e_machine = struct.unpack_from("<H", hdr, 18)[0]
            e_shoff = struct.unpack_from("<Q", hdr, 40)[0]
            e_shentsize, e_shnum = struct.unpack_from("<HH", hdr, 58)
            if e_machine == 224:  # EM_AMDGPU
                end = pos + e_shoff + e_shentsize * e_shnum
                out.append(data[pos:end])
                pos = data.find(b"\x7fELF", end)
                continue
        pos = data.find(b"\x7fELF", pos + 4)
    return out


def kernel_resources(lib: str = None) -> dict:
    """{kernel symbol: {field: int}} over every embedded code object"""
    lib = lib or os.path.join(ROOT, "opencv_amd", "lib", "libtbdk.so")
    data = open(lib, "rb").read()
    res = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(data)):
            p = os.path.join(d, f"co{i}.elf")
            with open(p, "wb") as fh:
                fh.write(co)
            txt = subprocess.run([READELF, "--notes", p], capture_output=True, text=True, check=True).stdout
            cur = {}
            for line in txt.splitlines():
                m = re.match(r"\s*-?\s*(\.[a-z_]+):\s+(\S+)", line)
                if not m:
                    continue
                key, val = m.group(1), m.group(2)
                if key == ".group_segment_fixed_size" and cur.get(".name"):
                    cur = {}
                if key in FIELDS:
                    cur[key] = int(val)
                elif key == ".name" and not val.startswith("."):
                    cur[".name"] = val
                    if all(f in cur for f in FIELDS):
                        res[val] = {f.lstrip("."): cur[f] for f in FIELDS}
                        cur = {}
                if ".name" in cur and all(f in cur for f in FIELDS):
                    res[cur[".name"]] = {f.lstrip("."): cur[f] for f in FIELDS}
                    cur = {}
    return res


def main(argv):
    res = kernel_resources(argv[1] if len(argv) > 1 else None)
    for k in sorted(res):
        r = res[k]
        print(f"lds {r['group_segment_fixed_size']:6d}  scratch {r['private_segment_fixed_size']:4d}  "
              f"vgpr {r['vgpr_count']:3d}  sgpr {r['sgpr_count']:3d}  spill {r['vgpr_spill_count']}/"
              f"{r['sgpr_spill_count']}  {k}")


if __name__ == "__main__":
    main(sys.argv)
