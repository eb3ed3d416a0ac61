#!/usr/bin/env python3
"""Vendor the reference-owned test fixtures the CPU suite reads into tests/fixtures/ (so no test depends on
/root/reference being present):
  * data files copied as they are: iris.dat, the ansj core dictionary, the kuromoji test resources, the Keras model
    import fixtures, the deeplearning4j-graph test graphs;
  * the numeric literals of three reference unit tests (SubsamplingLayerTest, ConvolutionLayerTest,
    LocalResponseTest): every ``Nd4j.create(new double[]{...}, new int[]{...})`` array with its source offset and the
    variable it is assigned to, plus the offsets of the method / field declarations the tests locate them by, as
    JSON (tests/fixtures/java/<Test>.json) — the Java sources themselves are not copied.
Usage: python tools/vendor_fixtures.py [--ref /root/reference]"""
import argparse
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "fixtures")
DATA = [
    "deeplearning4j-core/src/main/resources/iris.dat",
    "deeplearning4j-nlp-parent/deeplearning4j-nlp-chinese/src/main/resources/core.dic",
    "deeplearning4j-nlp-parent/deeplearning4j-nlp-japanese/src/test/resources",
    "deeplearning4j-modelimport/src/test/resources",
    "deeplearning4j-graph/src/test/resources",
]
JAVA = [
    "deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/convolution/SubsamplingLayerTest.java",
    "deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/convolution/ConvolutionLayerTest.java",
    "deeplearning4j-core/src/test/java/org/deeplearning4j/nn/layers/normalization/LocalResponseTest.java",
]
ARR = re.compile(r"(?:(\w+)\s*=\s*)?Nd4j\.create\(new double\[\]\s*\{([^}]*)\}\s*,\s*new int\[\]\s*\{([^}]*)\}")
DECL = re.compile(r"public\s+(?:static\s+)?[\w<>\[\]]+\s+(\w+)\s*\(")


def java_json(path):
    text = open(path).read()
    arrays = []
    for m in ARR.finditer(text):
        arrays.append({"pos": m.start(), "name": m.group(1),
                       "values": [float(v) for v in m.group(2).replace("\n", " ").split(",") if v.strip()],
                       "shape": [int(v) for v in m.group(3).split(",")]})
    decls = {}
    for m in DECL.finditer(text):
        decls.setdefault(m.group(1), m.start())
    return {"source": os.path.relpath(path, "/root/reference"), "arrays": arrays, "declarations": decls}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    for rel in DATA:
        src, dst = os.path.join(a.ref, rel), os.path.join(FIX, rel)
        if os.path.isdir(src):
            if os.path.exists(dst):
                shutil.rmtree(dst)
            shutil.copytree(src, dst)
        else:
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            shutil.copyfile(src, dst)
        for dp, _, fs in os.walk(dst if os.path.isdir(dst) else os.path.dirname(dst)):
            for f in fs:
                os.chmod(os.path.join(dp, f), 0o644)
    os.makedirs(os.path.join(FIX, "java"), exist_ok=True)
    for rel in JAVA:
        out = os.path.join(FIX, "java", os.path.basename(rel).replace(".java", ".json"))
        with open(out, "w") as fh:
            json.dump(java_json(os.path.join(a.ref, rel)), fh, indent=0)
    print("vendored into", FIX)


if __name__ == "__main__":
    main()
