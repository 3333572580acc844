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
      round-5 stage-split object lost the row index that way);
  P3  the register allocator's live-range split done inside any divergent
      region (an if / else arm up to its exec restore): `v_mov vA, vB` (or a
      spill store) with exec narrowed, undone by `v_mov vB, vA` (or a reload
      of the same slot) after exec is widened again -- the lanes outside the
      region get vA's stale contents back (the round-5 epoch-priority object
      corrupted its per-lane thread id that way and leaked arena chunks).

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


NARROW = re.compile(r"s_(and|andn2|or|xor)_saveexec_b64 |s_mov_b64 exec, s\[|s_xor_b64 exec, exec|"
                    r"s_andn2_b64 exec, exec|s_and_b64 exec, exec")


def _other_arm_writes(L, k, regs):
    """for an else arm starting at k (`s_andn2_saveexec_b64 sX, sX` / `s_or_saveexec_b64
    sX, sX`): does the matching if arm write any of regs?"""
    m = re.match(r"s_(andn2|or)_saveexec_b64 (s\[\d+:\d+\]), (s\[\d+:\d+\])$", L[k])
    if not m or m.group(2) != m.group(3):
        return False
    sx = re.escape(m.group(2))
    for t in range(k - 1, max(-1, k - 4000), -1):
        if re.match(r"s_(and_saveexec_b64 %s,|xor_b64 %s, exec, )" % (sx, sx), L[t]):
            for u in range(t + 1, k):
                d, _ = _dst_src(L[u])
                if d & regs:
                    return True
            return False
    return False


def check_split_copies(L):
    """P3: split copies made with exec narrowed and undone with it widened"""
    bad = []
    n = len(L)
    k = 0
    while k < n:
        if not NARROW.match(L[k]):
            k += 1
            continue
        j = k + 1
        while j < n and not ("exec" in L[j] or L[j].startswith(ENDS)):
            j += 1
        if j >= n or not RESTORE.match(L[j]):
            k = j if j > k else k + 1
            continue
        for i in range(k + 1, j):
            c = L[i]
            m = re.match(r"v_mov_b(32|64)_e32 (v\S+), (v\S+)$", c)
            sp = re.match(r"scratch_store_\S+ off, (v\S+), off offset:(\d+)", c)
            if m:
                a, b = m.group(2), m.group(3)
                if _other_arm_writes(L, k, _regs(a)):
                    continue   # a phi: the if-arm writes the register too
                undo = re.compile(r"v_mov_b%s_e32 %s, %s$" % (m.group(1), re.escape(b), re.escape(a)))
                for t in range(j + 1, min(n, j + 12000)):
                    if undo.match(L[t]):
                        bad.append((i + 1, c, "split under a narrowed exec (region %d-%d), undone at %d"
                                    % (k + 1, j + 1, t + 1)))
                        break
                    d, _ = _dst_src(L[t])
                    if d & _regs(a):
                        break
            elif sp:
                slot = sp.group(2)
                for t in range(j + 1, min(n, j + 12000)):
                    if re.match(r"scratch_load_\S+ \S+, off, off offset:%s\b" % slot, L[t]):
                        bad.append((i + 1, c, "spilled under a narrowed exec (region %d-%d), reloaded at %d"
                                    % (k + 1, j + 1, t + 1)))
                        break
                    if re.match(r"scratch_store_\S+ off, \S+, off offset:%s\b" % slot, L[t]):
                        break
        k = j
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
    seen = {b[0] for b in bad}
    return bad + check_loop_exits(L) + [b for b in check_split_copies(L) if b[0] not in seen]


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


ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
LLVM = os.path.join(ROCM, "lib", "llvm", "bin") + "/"
ARCH = os.environ.get("ARCH", "gfx950")   # the Makefile's ARCH


def disassemble(path):
    """ARCH disassembly of the device code bundled in a host .so / .o (a
    linked library's .hip_fatbin holds one offload bundle per object file,
    plain or compressed), or None when no code object for ARCH can be taken
    out of it (another target, a bundle format these tools do not read): the
    caller reports the file as not checked instead of failing the build."""
    d = tempfile.mkdtemp()
    fb = os.path.join(d, "fb")
    r = subprocess.run([LLVM + "llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, path,
                        os.path.join(d, "x")], stderr=subprocess.DEVNULL)
    if r.returncode != 0 or not os.path.exists(fb):
        return None
    data = open(fb, "rb").read()
    magics = (b"__CLANG_OFFLOAD_BUNDLE__", b"CCOB")
    starts = sorted(m.start() for mg in magics for m in re.finditer(re.escape(mg), data))
    out = []
    for i, st in enumerate(starts):
        piece, co = os.path.join(d, "b%d" % i), os.path.join(d, "co%d" % i)
        open(piece, "wb").write(data[st:starts[i + 1] if i + 1 < len(starts) else len(data)])
        r = subprocess.run([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", "--input=" + piece,
                            "--targets=hipv4-amdgcn-amd-amdhsa--" + ARCH, "--output=" + co],
                           stderr=subprocess.DEVNULL)
        if r.returncode == 0 and os.path.exists(co) and os.path.getsize(co):
            dis = subprocess.run([LLVM + "llvm-objdump", "-d", "--mcpu=" + ARCH, co],
                                 capture_output=True, text=True)
            if dis.returncode == 0:
                out.append(dis.stdout)
    return "\n".join(out) if out else None


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
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-fvisibility=hidden", "-std=c++17", "--offload-arch=" + ARCH,
           "--offload-device-only",
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
        if text is None:
            print("%s: not checked (no %s code object could be extracted)" % (os.path.basename(fn), ARCH))
            continue
        bad += check_text(text, os.path.basename(fn))
    sys.exit(1 if bad else 0)
