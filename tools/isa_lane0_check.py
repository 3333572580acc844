"""Static check of the GPU code objects for the code-generation pattern behind
the diagnostic builds' K3 stalls: register copies of
wave-wide values that the compiler placed where the wave runs with only some
lanes, or none, enabled:

  P1  vector instructions between a divergent loop's exit (`s_andn2_b64 exec,
      exec, ..` + `s_cbranch_execnz`) and the next exec-mask change: they run
      with EXEC = 0, i.e. do nothing (the round-5 trace+check object copied
      the row-wavefront word's address there and then polled a stale one);
  P2  a copy or spill of a value defined outside a lane-masked region (a
      hoisted lane mask, `s_mov_b64 exec, s[..]` ... `s_or_b64 exec, exec,
      s[..]`: the code of `if (tid == 0) ...`) whose destination is read with
      the full mask afterwards, so 63 lanes read a stale register (the
      round-5 stage-split object lost the row index that way).

usage: python tools/isa_lane0_check.py <device .s | .so | .o> [...]
       python tools/isa_lane0_check.py --build [-D...]   (compiles vp8_k3.hip for gfx950)
Exit status 1 if any function has either pattern."""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RESTORE = re.compile(r"s_or_b64 exec, exec, ")
ENDS = ("s_cbranch", "s_branch", "s_andn2_b64 exec", ".LBB", "s_setpc", "s_endpgm")


def _regs(s):
    r = set()
    for m in re.finditer(r"v\[(\d+):(\d+)\]", s):
        r |= set(range(int(m.group(1)), int(m.group(2)) + 1))
    for m in re.finditer(r"\bv(\d+)\b", s):
        r.add(int(m.group(1)))
    return r


def _dst_src(c):
    parts = c.split(None, 1)
    if len(parts) < 2:
        return set(), set()
    op, args = parts
    a = [x.strip() for x in re.split(r",(?![^\[]*\])", args)]
    if op.startswith(("ds_write", "global_store", "scratch_store", "buffer_store")) or \
            (op.startswith(("ds_", "global_atomic")) and "rtn" not in op and "read" not in op):
        return set(), _regs(args)
    if op.startswith("s_") or op.startswith(("v_readlane", "v_readfirstlane")) or \
            (op.startswith("v_cmp") and "_e64" not in op):
        return set(), _regs(args)
    if op.startswith("v_cmp"):
        return set(), _regs(",".join(a[1:]))
    return _regs(a[0]), _regs(",".join(a[1:]))


def _masked_spans(L):
    """[start, end) line spans of lane-masked regions (hoisted masks)"""
    spans = []
    k = 0
    while k < len(L):
        if re.match(r"s_mov_b64 exec, s\[\d+:\d+\]$", L[k]):
            j = k + 1
            while j < len(L) and not (RESTORE.match(L[j]) or L[j].startswith(ENDS) or
                                      L[j].startswith("s_mov_b64 exec") or "saveexec" in L[j]):
                j += 1
            if j < len(L) and RESTORE.match(L[j]):
                spans.append((k, j))
            k = j
        else:
            k += 1
    return spans


def check_loop_exits(L):
    """P1: vector work after a divergent loop's exit, before EXEC is restored"""
    bad = []
    for k in range(len(L) - 1):
        if not re.match(r"s_andn2_b64 exec, exec, ", L[k]):
            continue
        j = k + 1
        while j < len(L) and not L[j]:
            j += 1
        if j >= len(L) or not L[j].startswith("s_cbranch_execnz"):
            continue
        t = j + 1
        while t < len(L):
            c = L[t]
            if not c:
                t += 1
                continue
            if "exec" in c or c.startswith(ENDS):
                break
            if not c.startswith(("s_", ".", "v_readlane", "v_readfirstlane", "v_writelane")):
                bad.append((t + 1, c, "runs with EXEC = 0 after the loop at %d" % (k + 1)))
            t += 1
    return bad


def check_function(lines):
    L = [ln.split(";")[0].split("//")[0].strip() for ln in lines]
    spans = _masked_spans(L)
    inside = [False] * len(L)
    for s, e in spans:
        for i in range(s, e):
            inside[i] = True
    bad = []
    for s, e in spans:
        written = set()
        for i in range(s + 1, e):
            c = L[i]
            if not c or c.startswith("."):
                continue
            m = re.match(r"v_mov_b(?:32|64)_e32 (v\S+), (v\S+)$", c)
            sp = re.match(r"scratch_store_\S+ off, (v\S+),", c)
            src = m.group(2) if m else (sp.group(1) if sp else None)
            if src and not (_regs(src) & written):
                if sp:
                    bad.append((i + 1, c, "spill store of a wave-wide value under a lane mask"))
                else:
                    dst = _regs(m.group(1))
                    for t in range(e + 1, min(len(L), e + 6000)):
                        d, r = _dst_src(L[t])
                        if dst & r:
                            if not inside[t] and not L[t].startswith(("v_readlane", "v_readfirstlane")):
                                bad.append((i + 1, c, "read with the full mask at %d: %s" % (t + 1, L[t])))
                            break
                        if dst & d:
                            break
            d, _ = _dst_src(c)
            written |= d
    return bad + check_loop_exits(L)


def functions(text):
    cur, buf = None, []
    for ln in text.splitlines():
        m = re.match(r"^(_Z\S+):", ln) or re.match(r"^[0-9a-f]+ <(\S+)>:", ln)
        if m:
            if cur:
                yield cur, buf
            cur, buf = m.group(1), []
            continue
        if cur:
            if ln.startswith(".Lfunc_end"):
                yield cur, buf
                cur = None
            else:
                buf.append(ln)
    if cur:
        yield cur, buf


LLVM = "/opt/rocm/lib/llvm/bin/"


def disassemble(path):
    """gfx950 disassembly of the device code bundled in a host .so / .o"""
    d = tempfile.mkdtemp()
    fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
    subprocess.run([LLVM + "llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, path, os.path.join(d, "x")],
                   check=True, stderr=subprocess.DEVNULL)
    subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fb,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co], check=True)
    return subprocess.run([LLVM + "llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                          capture_output=True, text=True).stdout


def check_text(text, label):
    n = 0
    for name, body in functions(text):
        for ln, c, why in check_function(body):
            n += 1
            if n <= 20:
                print("%s: %s line %d: %s  (%s)" % (label, name[:48], ln, c, why))
    print("%s: %d copies under a partial or empty lane mask" % (label, n))
    return n


def build_asm(flags):
    src = os.path.join(ROOT, "libwebp_amd", "csrc", "hip", "vp8_k3.hip")
    out = os.path.join(tempfile.mkdtemp(), "k3.s")
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only",
           "-Wno-unused-result", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(ROOT, "libwebp_amd", "csrc"), "-S", src, "-o", out] + flags
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--build":
        flags = sys.argv[2:]
        sys.exit(1 if check_text(build_asm(flags), "vp8_k3 " + " ".join(flags)) else 0)
    bad = 0
    for fn in sys.argv[1:]:
        text = disassemble(fn) if fn.endswith((".so", ".o")) else open(fn).read()
        bad += check_text(text, os.path.basename(fn))
    sys.exit(1 if bad else 0)
