"""Extracts the two trained linear-SVM people detectors the reference ships as
float tables into little-endian float32 files under opencv_amd/data/:

  hog_people_64x128.f32  HOGDescriptor::getDefaultPeopleDetector()
                         (objdetect/src/hog.cpp:2174-2984; the same table as
                         cudaobjdetect/src/hog.cpp:1031 getPeopleDetector64x128)
  hog_people_48x96.f32   HOGDescriptor::getDaimlerPeopleDetector()
                         (objdetect/src/hog.cpp:2987-3487; = cudaobjdetect's
                         getPeopleDetector48x96, cudaobjdetect/src/hog.cpp:693)

These are model coefficients (data), needed for getDefaultPeopleDetector().
Run here, where /root/reference exists; the outputs are committed.  The float
literals are converted by gcc (a temporary C file), so each one rounds exactly
as the reference's compiler rounds it."""
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference/modules/objdetect/src/hog.cpp"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "opencv_amd", "data")


def table(text, func):
    i = text.index(func)
    a = text.index("{", text.index("detector[]", i)) + 1
    b = text.index("}", a)
    toks = re.findall(r"[-+]?(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?f?", text[a:b])
    return [t if t.endswith("f") else t + "f" for t in toks]


def to_f32(toks):
    with tempfile.TemporaryDirectory() as d:
        src, exe, out = os.path.join(d, "t.c"), os.path.join(d, "t"), os.path.join(d, "o.bin")
        with open(src, "w") as f:
            f.write("#include <stdio.h>\nstatic const float v[] = {%s};\n" % ",".join(toks))
            f.write('int main(int c, char** a){FILE* o=fopen(a[1],"wb");'
                    'fwrite(v,4,sizeof v/4,o);fclose(o);return 0;}\n')
        subprocess.run(["gcc", "-O0", src, "-o", exe], check=True)
        subprocess.run([exe, out], check=True)
        return np.fromfile(out, "<f4")


def main():
    text = open(REF).read()
    os.makedirs(OUT, exist_ok=True)
    for func, name, n in (("HOGDescriptor::getDefaultPeopleDetector()", "hog_people_64x128.f32", 3781),
                          ("HOGDescriptor::getDaimlerPeopleDetector()", "hog_people_48x96.f32", 1981)):
        v = to_f32(table(text, func))
        assert v.size == n, (name, v.size)
        v.astype("<f4").tofile(os.path.join(OUT, name))
        print(name, v.size, v[:3], v[-1])


if __name__ == "__main__":
    sys.exit(main())
