"""Static checks on the gfx950 code objects inside libccmi.so (CPU only: llvm-objdump).

The LDS-DMA pieces of the k-means and co-association kernels are issued from inline asm that
loads M0 itself (`s_mov_b32 m0, sN` + `global_load_lds_*`, kmeans.hip / coassoc.hip dma16).  The
AMDGPU backend treats M0 as a reserved register, so an "m0" clobber is ignored (the compiler
warns); what keeps the asm safe is that no compiler-generated code relies on M0 across it.  That
is checked here on the ISA instead of assumed: every instruction naming M0 is our
`s_mov_b32 m0` directly followed by an LDS-DMA load, every LDS-DMA load directly follows one, and
no instruction that reads M0 implicitly (movrel, sendmsg, GWS, append/consume, interpolation)
appears at all."""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "consensus_clustering_amd",
                   "libccmi.so")
IMPLICIT_M0 = ("movrel", "s_sendmsg", "ds_gws", "ds_append", "ds_consume", "v_interp", "lds_param_load",
               "s_ttracedata")


def _code_objects(tmp_path):
    fb = tmp_path / "fatbin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", LIB, str(tmp_path / "lib.so")],
                   check=True, capture_output=True)
    data = fb.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    offs = [m.start() for m in re.finditer(re.escape(magic), data)]
    assert offs, "no offload bundles in .hip_fatbin"
    for k, o in enumerate(offs):
        piece = tmp_path / f"b{k}"
        piece.write_bytes(data[o:offs[k + 1] if k + 1 < len(offs) else len(data)])
        co = tmp_path / f"b{k}.co"
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={piece}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                       capture_output=True)
        out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", str(co)], check=True,
                             capture_output=True, text=True).stdout
        ins = []
        for line in out.splitlines():
            line = line.split("//")[0].strip()
            if line and not line.endswith(":") and not line.startswith("Disassembly"):
                ins.append(line)
        yield k, ins


@pytest.mark.skipif(not (os.path.exists(LIB) and shutil.which(f"{LLVM}/llvm-objdump")),
                    reason="libccmi.so or the ROCm llvm tools are missing")
def test_m0_is_only_set_by_the_lds_dma_asm(tmp_path):
    seen = 0
    for k, ins in _code_objects(tmp_path):
        for i, l in enumerate(ins):
            op = l.split()[0]
            assert not any(t in op for t in IMPLICIT_M0), (k, l)
            if re.search(r"\bm0\b", l):
                assert re.fullmatch(r"s_mov_b32 m0, s\d+", l), (k, l)
                assert i + 1 < len(ins) and ins[i + 1].startswith("global_load_lds"), (k, l, ins[i + 1])
                seen += 1
            if op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in l):
                assert i > 0 and re.fullmatch(r"s_mov_b32 m0, s\d+", ins[i - 1]), (k, ins[i - 1], l)
    assert seen > 0, "no LDS-DMA asm found: the check no longer looks at the kernels it guards"
