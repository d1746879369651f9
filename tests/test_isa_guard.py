"""CPU: guards on the machine code of the built libore.so (gfx950), read with the ROCm binutils from the
library's offload bundle; no kernel runs.

The band walker (conv_band_pool_f32_kernel, ore_conv1_f32.hip) takes the pooled neighbour column of a
lane from lane l + 1 by a DPP wave_shl:1 read with bound_ctrl (an out-of-range source reads 0).  A DPP
read returns 0 from a source lane that EXEC disables, so the exchange is only right while every lane of
the wave executes it.  Round 5 saw a restructured epilogue give wrong pooled maxima (VERDICT r05 item 2,
DESIGN.md 3.4b); this test pins the properties the product relies on, so that an edit which moves the
exchange under divergent control flow fails here, on the CPU, before it can reach the GPU tests."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import ore
from ore import _lib

LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
OBJDUMP = os.path.join(LLVM, "llvm-objdump")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _tools():
    return os.path.exists(BUNDLER) and os.path.exists(OBJDUMP) and shutil.which("objcopy")


def _kernel_isa(symbol_part):
    """Disassembly lines of the first kernel whose symbol contains symbol_part."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", _lib.LIB_PATH, fat], check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for i in range(len(starts) - 1):
            part = os.path.join(d, f"b{i}.bin")
            open(part, "wb").write(data[starts[i]:starts[i + 1]])
            elf = os.path.join(d, f"b{i}.elf")
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(elf):
                continue
            dis = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", elf], capture_output=True, text=True).stdout
            lines, on = [], False
            for ln in dis.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.*)>:", ln)
                if m:
                    if on:
                        return lines
                    on = symbol_part in m.group(1)
                    continue
                if on and ln.startswith("\t"):
                    ins = ln.strip().split("//")[0].strip()
                    if ins:
                        lines.append(ins)
            if on:
                return lines
    return None


@pytest.mark.skipif(not _tools(), reason="ROCm binutils / objcopy not present")
@pytest.mark.parametrize("kernel,group", [
    ("conv_band_pool_f32_kernel", 16),  # 16 channel rows per 32-channel fragment, 3 fragments per step
    ("conv_band_pool_f16_kernel", 4),   # round 6: 4 f16 channel pairs per (fragment, group), 6 per row
])
def test_band_walker_dpp_exchange_runs_with_full_exec(kernel, group):
    ore.load()
    isa = _kernel_isa(kernel)
    assert isa, f"{kernel} not found in libore.so"
    dpp = [k for k, i in enumerate(isa) if "wave_shl:1" in i]
    # (the compiler may duplicate the step)
    assert dpp and len(dpp) % group == 0, len(dpp)
    for k in dpp:
        ins = isa[k]
        # all rows and banks written, an out-of-range source (lane 63) reads 0
        assert "row_mask:0xf" in ins and "bank_mask:0xf" in ins and "bound_ctrl:1" in ins, ins
        # the last instruction before it that writes EXEC restores it (the end of a divergent region); an
        # s_and_saveexec / s_and / s_andn2 of exec here would mean the exchange runs EXEC-masked
        last = next((isa[j] for j in range(k - 1, -1, -1) if re.match(r"s_\w+ exec, ", isa[j])
                     or "saveexec" in isa[j]), None)
        assert last is None or re.match(r"s_(or|mov)_b64 exec, ", last), (ins, last)
        # the DPP's source VGPR was last written by a single-register (32-bit) definition: ROCm 7.2's compiler
        # lowers a DPP of either half of a packed f32 pair (a v_pk_* result, v[n:n+1]) as a DPP of the LOW half
        # and uses it for both (tests/test_isa_guard.py::test_compiler_dpp_packed_pair_hazard)
        src = int(re.match(r"v_\w+_dpp v\d+, v(\d+)", ins).group(1))
        for jj in range(k - 1, -1, -1):
            d = isa[jj].split()
            if len(d) < 2 or not d[0].startswith("v_") or d[0].startswith("v_cmp"):
                continue
            dst = d[1].rstrip(",")
            m1 = re.fullmatch(r"v(\d+)", dst)
            m2 = re.fullmatch(r"v\[(\d+):(\d+)\]", dst)
            if m1 and int(m1.group(1)) == src:
                break
            if m2 and int(m2.group(1)) <= src <= int(m2.group(2)):
                raise AssertionError(f"DPP source v{src} last written by a multi-register definition: {isa[jj]} -> {ins}")


@pytest.mark.skipif(not _tools(), reason="ROCm binutils / objcopy not present")
def test_compiler_dpp_packed_pair_hazard(tmp_path):
    """Pins the compiler behaviour the guard above avoids (ROCm 7.2, gfx950): a DPP of each half of a packed f32
    sum compiles to ONE v_mov_b32_dpp of the low half, used for both halves -- wrong values for the high half.
    If a future compiler fixes it this test fails, and the note in DESIGN.md 3.4b can go."""
    src = tmp_path / "r.hip"
    src.write_text("""#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
extern "C" __global__ void k(const f2* a, const f2* b, float* out) {
  const f2 v = a[threadIdx.x] + b[threadIdx.x];
  for (int q = 0; q < 2; ++q)
    out[2 * threadIdx.x + q] = fmaxf(v[q], __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
        0, __builtin_bit_cast(int, v[q]), 0x130, 0xf, 0xf, true)));
}
""")
    out = tmp_path / "r.s"
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", "-o", str(out),
                        str(src)], capture_output=True, text=True)
    if r.returncode != 0 or not out.exists():
        pytest.skip("hipcc not usable here")
    asm = out.read_text()
    assert "v_pk_add_f32" in asm
    assert asm.count("_dpp") == 1, asm.count("_dpp")  # two values shifted, one DPP: the miscompile


def _kernel_meta():
    """{kernel name: {vgpr_count, agpr_count, private_segment_fixed_size, group_segment_fixed_size}} from the gfx950
    code object's AMDGPU metadata note (llvm-readelf --notes)."""
    readelf = os.path.join(LLVM, "llvm-readelf")
    meta = {}
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", _lib.LIB_PATH, fat], check=True)
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for i in range(len(starts) - 1):
            part = os.path.join(d, f"b{i}.bin")
            open(part, "wb").write(data[starts[i]:starts[i + 1]])
            elf = os.path.join(d, f"b{i}.elf")
            r = subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={elf}"], capture_output=True)
            if r.returncode != 0 or not os.path.exists(elf):
                continue
            notes = subprocess.run([readelf, "--notes", elf], capture_output=True, text=True).stdout
            for entry in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
                name = re.search(r"\.name:\s+(\S+)", entry)
                if not name:
                    continue
                row = {"agpr_count": int(entry.split("\n", 1)[0].strip() or 0)}
                for key in ("vgpr_count", "private_segment_fixed_size", "group_segment_fixed_size"):
                    m = re.search(r"\." + key + r":\s+(\d+)", entry)
                    row[key] = int(m.group(1)) if m else 0
                meta[name.group(1)] = row
    return meta


@pytest.mark.skipif(not _tools() or not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                    reason="ROCm binutils / objcopy not present")
def test_pooled_squeeze_occupancy():
    """Round 6: the fire4 -> pool3 -> fire5 instance of the pooled squeeze with e1 inside (KS1 = 8, SPLIT = 2) runs
    three waves per SIMD (230 -> 210 us against two).  A unified register file of 512 per lane gives
    three waves at <= 168 registers (the metadata's vgpr_count, AGPRs included); an edit or a compiler that needs more drops it back to two.
    The plain pool5 instance keeps its six waves; the Winograd LDS kernel its two (two workgroups per CU)."""
    ore.load()
    meta = _kernel_meta()
    assert meta, "no kernel metadata in libore.so"

    def regs(part):
        rows = [v for k, v in meta.items() if part in k]
        assert rows, part
        return max(r["vgpr_count"] for r in rows)  # the unified count: arch VGPRs + AGPRs (granule 8)

    assert regs("pool_conv1x1_f32_kernelILi2ELi8ELi6ELi2E") <= 168
    assert regs("pool_conv1x1_f32_kernelILi1ELi0ELi0ELi1E") <= 512 // 6 // 8 * 8
    assert regs("conv_winol_kernel") <= 256
