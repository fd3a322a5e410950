#!/usr/bin/env python3
"""Build the native parts of wormhole_amd in-tree (gfx950 only).

Two shared objects are produced next to the Python sources:

* ``wormhole_amd/_hip.so``  -- hand-written CDNA4 HIP kernels (``csrc/hip/*.hip``,
  compiled by ``hipcc --offload-arch=gfx950`` WITHOUT torch headers so each
  kernel file builds in seconds) plus the torch/pybind11 binding layer
  (``csrc/bind/*.cc``, host-only g++ compile that validates tensors and
  launches on the current HIP stream).
* ``bin/native/{convert,text2crb}`` -- standalone C++ data conversion tools
  (reference learn/tool/), wrapped by ``bin/convert.dmlc`` / ``bin/text2crb.dmlc``.
* ``wormhole_amd/_host.so`` -- the native C++ runtime (``csrc/host/*.cc``):
  proto-text config parser, data parsers (libsvm / criteo / adfea / crb),
  CityHash64, LZ4 block codec, RecordIO, workload pool, control-plane
  sockets, CPU localizer.  Host-only, no GPU needed.

A ``build/build.ninja`` is generated and driven by ninja so rebuilds are
incremental and parallel.  Usage: ``python build_native.py [-j N] [--clean]``.
"""
import argparse
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(ROOT, "build")
PKG = os.path.join(ROOT, "wormhole_amd")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"


def torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths()
    lib = ce.library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def gen_ninja():
    inc, tlib, abi = torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    common_inc = "-I%s/csrc" % ROOT
    tinc = " ".join("-isystem %s" % p for p in inc) + " -isystem %s" % pyinc
    cxxflags = ("-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-sign-compare "
                "-D_GLIBCXX_USE_CXX11_ABI=%d %s" % (abi, common_inc))
    hipflags = ("-O3 -std=c++17 -fPIC --offload-arch=%s -munsafe-fp-atomics "
                "-Wno-unused-result %s" % (ARCH, common_inc))
    bindflags = ("%s -D__HIP_PLATFORM_AMD__ -DUSE_ROCM -isystem %s/include %s "
                 "-DTORCH_API_INCLUDE_EXTENSION_H" % (cxxflags, ROCM, tinc))
    hostflags = "%s %s -DTORCH_API_INCLUDE_EXTENSION_H -pthread" % (cxxflags, tinc)
    tlibs = "-L%s -Wl,-rpath,%s -lc10 -ltorch -ltorch_cpu -ltorch_python" % (tlib, tlib)
    hiplibs = "%s -lc10_hip -ltorch_hip -lamdhip64 -lrccl" % tlibs

    lines = [
        "ninja_required_version = 1.3",
        "hipcc = %s" % hipcc,
        "cxx = g++",
        "rule hip",
        "  command = $hipcc %s -MD -MF $out.d -c $in -o $out" % hipflags,
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = HIPCC $in",
        "rule bind",
        "  command = $cxx %s -MD -MF $out.d -c $in -o $out" % bindflags,
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(bind) $in",
        "rule host",
        "  command = $cxx %s -MD -MF $out.d -c $in -o $out" % hostflags,
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(host) $in",
        "rule link_hip",
        "  command = $hipcc --offload-arch=%s -shared -fPIC $in -o $out %s" % (ARCH, hiplibs),
        "  description = LINK $out",
        "rule link_host",
        "  command = $cxx -shared -fPIC -pthread $in -o $out %s -lssl -lcrypto" % tlibs,
        "  description = LINK $out",
        "rule tool",
        "  command = $cxx -O3 -std=c++17 -Wall -Wno-sign-compare -pthread -I%s/csrc -MD -MF $out.d -c $in -o $out" % ROOT,
        "  depfile = $out.d",
        "  deps = gcc",
        "  description = CXX(tool) $in",
        "rule link_tool",
        "  command = $cxx -pthread $in -o $out -lssl -lcrypto",
        "  description = LINK $out",
    ]
    hip_objs = []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/hip/*.hip"))):
        obj = os.path.join(BUILD, "hip", os.path.basename(src) + ".o")
        lines.append("build %s: hip %s" % (obj, src))
        hip_objs.append(obj)
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/bind/*.cc"))):
        obj = os.path.join(BUILD, "bind", os.path.basename(src) + ".o")
        lines.append("build %s: bind %s" % (obj, src))
        hip_objs.append(obj)
    host_objs = []
    for src in sorted(glob.glob(os.path.join(ROOT, "csrc/host/*.cc"))):
        obj = os.path.join(BUILD, "host", os.path.basename(src) + ".o")
        lines.append("build %s: host %s" % (obj, src))
        host_objs.append(obj)
    # standalone native tools (no torch): bin/native/{convert,text2crb}
    core = []
    for name in ("parsers", "io", "remote_fs", "json", "lz4", "cityhash"):
        obj = os.path.join(BUILD, "tool", name + ".o")
        lines.append("build %s: tool %s" % (obj, os.path.join(ROOT, "csrc/host/%s.cc" % name)))
        core.append(obj)
    lib = os.path.join(BUILD, "tool", "convert_lib.o")
    lines.append("build %s: tool %s" % (lib, os.path.join(ROOT, "csrc/tools/convert_lib.cc")))
    core.append(lib)
    for tool in ("convert", "text2crb"):
        obj = os.path.join(BUILD, "tool", tool + ".o")
        lines.append("build %s: tool %s" % (obj, os.path.join(ROOT, "csrc/tools/%s.cc" % tool)))
        lines.append("build %s: link_tool %s %s" % (os.path.join(ROOT, "bin", "native", tool), obj,
                                                    " ".join(core)))
    # host runtime self-test (no torch): bin/native/host_selftest
    st = []
    for name in ("workload_pool", "conf_parser", "van"):
        obj = os.path.join(BUILD, "tool", name + ".o")
        lines.append("build %s: tool %s" % (obj, os.path.join(ROOT, "csrc/host/%s.cc" % name)))
        st.append(obj)
    obj = os.path.join(BUILD, "tool", "host_selftest.o")
    lines.append("build %s: tool %s" % (obj, os.path.join(ROOT, "csrc/tests/host_selftest.cc")))
    lines.append("build %s: link_tool %s %s %s" % (
        os.path.join(ROOT, "bin", "native", "host_selftest"), obj, " ".join(st),
        " ".join(o for o in core if not o.endswith("convert_lib.o"))))
    lines.append("build %s: link_hip %s" % (os.path.join(PKG, "_hip.so"), " ".join(hip_objs)))
    lines.append("build %s: link_host %s" % (os.path.join(PKG, "_host.so"), " ".join(host_objs)))
    os.makedirs(BUILD, exist_ok=True)
    with open(os.path.join(BUILD, "build.ninja"), "w") as f:
        f.write("\n".join(lines) + "\n")


SELFTEST_SRCS = ("csrc/tests/host_selftest.cc", "csrc/host/parsers.cc", "csrc/host/io.cc",
                 "csrc/host/remote_fs.cc", "csrc/host/lz4.cc", "csrc/host/cityhash.cc", "csrc/host/workload_pool.cc",
                 "csrc/host/conf_parser.cc", "csrc/host/van.cc", "csrc/host/json.cc")


def build_sanitized(kind, jobs=None):
    """The host self-test under -fsanitize=<kind> (address | thread |
    undefined), host code only: build/san-<kind>/host_selftest."""
    out_dir = os.path.join(BUILD, "san-" + kind)
    os.makedirs(out_dir, exist_ok=True)
    flags = ["-O1", "-g", "-std=c++17", "-pthread", "-fno-omit-frame-pointer",
             "-fsanitize=" + kind, "-I" + os.path.join(ROOT, "csrc")]
    objs = []
    for src in SELFTEST_SRCS:
        obj = os.path.join(out_dir, os.path.basename(src) + ".o")
        subprocess.run(["g++"] + flags + ["-c", os.path.join(ROOT, src), "-o", obj], check=True)
        objs.append(obj)
    exe = os.path.join(out_dir, "host_selftest")
    subprocess.run(["g++"] + flags + objs + ["-o", exe, "-lssl", "-lcrypto"], check=True)
    return exe


def build(jobs=None, clean=False, verbose=False):
    if clean and os.path.isdir(BUILD):
        shutil.rmtree(BUILD)
    gen_ninja()
    jobs = jobs or min(16, os.cpu_count() or 4)
    cmd = ["ninja", "-C", BUILD, "-j", str(jobs)]
    if verbose:
        cmd.append("-v")
    r = subprocess.run(cmd)
    if r.returncode != 0:
        raise SystemExit("native build failed (exit %d)" % r.returncode)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-v", action="store_true")
    ap.add_argument("--sanitize", choices=["address", "thread", "undefined"], default=None,
                    help="build the host self-test under a sanitizer instead")
    a = ap.parse_args()
    if a.sanitize:
        print(build_sanitized(a.sanitize, a.j))
        sys.exit(0)
    build(a.j, a.clean, a.v)
    sys.exit(0)
