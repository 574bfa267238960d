#!/usr/bin/env python3
"""Generate a bit-exact C/HIP restatement of glibc 2.35 libm's FMA-variant
``tan``, ``cos`` and ``log`` (x86_64 ifunc targets ``__tan_fma``, ``__cos_fma``,
``__log_fma``) from the system libm's machine code.

Why: the reference projects latitudes with CPython ``math.tan/cos/log``
(reference ``tile.py:17``), i.e. glibc libm.  glibc 2.35 is *not* correctly
rounded (measured here: ~0.27% of tan, ~0.17% of cos and ~0.09% of log
results differ from the correctly rounded value), so a GPU kernel that wants
the reference's exact tile row for points that sit within ~1e-13 of a tile
boundary has to reproduce glibc's own arithmetic, operation for operation.
The device slow path (``hm_exact_row`` in ``hm_project.h``) calls the functions
generated here; the fast path never does.

How: ``llvm-objdump`` disassembles each function; every instruction of the
small x86 subset these three functions use is restated as one C statement on
64-bit integer "registers" and double "xmm registers" (low lane only).  FMA
instructions become ``fma()``, every other float op a single IEEE op, so the
emitted code is exact on any IEEE-754 binary64 machine with a correct fma and
correctly rounded division -- gfx950 included.  Control flow keeps the
original branch structure as labels/gotos.  Constants and tables are copied
from libm's ``.rodata`` (they are data, not code).  The calls into
``__branred`` (Payne-Hanek reduction for |x| >= 105414350) go to the
hand-written restatement in ``heatmap_amd/csrc/hm_branred.h``.

The output header is committed; re-run this script only if libm changes:
    python tools/glibc_emul/gen_glibc_emul.py > heatmap_amd/csrc/hm_glibc_emul.h
``tests/test_math_host.py::test_glibc_restatement_bit_exact`` checks the generated code against the live libm
on millions of inputs on every CPU test run.
"""
import re
import struct
import subprocess
import sys

LIBM = "/lib/x86_64-linux-gnu/libm.so.6"
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# (name, start, stop) of the FMA ifunc targets in glibc 2.35-0ubuntu3.11 libm.
# Found from the IRELATIVE resolvers of tan/cos/__ieee754_log.
FUNCS = [
    ("log", 0x76660, 0x768B0),
    ("cos", 0x791C0, 0x799D0),
    ("tan", 0x799D0, 0x7A250),
]
# Tables addressed through a base register (leaq), with their byte sizes.
TABLES = {
    0xAEB80: 440 * 8,       # __sincostab (s_sin.c)
    0xB01E0: 0x90 + 128 * 16,  # __log_data (ln2hi, ln2lo, poly, poly1, tab)
    0xC15C0: 186 * 32,      # tan reduction table {x_i, F_i, G_i, ...}
}
# External targets: jumps/calls leaving the function.
EXTERN = {
    0x6F180: "branred",
    0x70A50: "math_invalid",
    0x70A20: "math_divzero",
    0xE240: "stack_chk_fail",
}

with open(LIBM, "rb") as f:
    IMAGE = f.read()


def rodata_u64(addr):
    return struct.unpack_from("<Q", IMAGE, addr)[0]


def hexd(u):
    """C hex-float literal of the double with bit pattern u (exact)."""
    d = struct.unpack("<d", struct.pack("<Q", u))[0]
    if d != d or d in (float("inf"), float("-inf")):
        return None
    return float.hex(d)


GPR64 = ["rax", "rbx", "rcx", "rdx", "rsi", "rdi", "rbp", "rsp", "r8", "r9",
         "r10", "r11", "r12", "r13", "r14", "r15"]
ALIAS = {}
for r in ["ax", "bx", "cx", "dx"]:
    ALIAS["r" + r] = ("r" + r, 64)
    ALIAS["e" + r] = ("r" + r, 32)
    ALIAS[r[0] + "l"] = ("r" + r, 8)
    ALIAS[r[0] + "h"] = ("r" + r, "h")
for r in ["si", "di", "bp"]:
    ALIAS["r" + r] = ("r" + r, 64)
    ALIAS["e" + r] = ("r" + r, 32)
    ALIAS[r + "l"] = ("r" + r, 8)
for n in range(8, 16):
    ALIAS["r%d" % n] = ("r%d" % n, 64)
    ALIAS["r%dd" % n] = ("r%d" % n, 32)


class Tr:
    def __init__(self, name, start, stop):
        self.name = name
        self.start = start
        self.lines = []
        out = subprocess.check_output(
            [OBJDUMP, "-d", "--no-show-raw-insn", "--start-address=%#x" % start,
             "--stop-address=%#x" % stop, LIBM], text=True)
        for ln in out.splitlines():
            mc = re.match(r"^\s*#\s*(0x[0-9a-f]+)\s*$", ln)
            if mc and self.lines:
                a, mn, r, c = self.lines[-1]
                self.lines[-1] = (a, mn, r, c + " # " + mc.group(1))
                continue
            m = re.match(r"\s*([0-9a-f]+):\s+(\S+)\s*(.*)$", ln)
            if not m:
                continue
            addr = int(m.group(1), 16)
            mnem = m.group(2)
            rest = m.group(3)
            comment = ""
            if "#" in rest:
                rest, comment = rest.split("#", 1)
            self.lines.append((addr, mnem, rest.strip(), comment.strip()))
        self.consts = {}
        self.used_tables = set()
        self.ptrbase = {}      # reg -> table base address (symbolic)
        self.lea_stack = {}    # reg -> stack slot whose address a leaq put there (__branred arguments)
        self.flags = None      # description of last flag-setting insn
        self.targets = set()
        for (a, mn, ops, c) in self.lines:
            if mn.startswith("j") and mn != "jmp" or mn == "jmp":
                t = ops.split()[0]
                if t.startswith("0x"):
                    self.targets.add(int(t, 16))
        self.out = []

    # ---- operand helpers -------------------------------------------------
    def split_ops(self, s):
        ops, depth, cur = [], 0, ""
        for ch in s:
            if ch == "(":
                depth += 1
            if ch == ")":
                depth -= 1
            if ch == "," and depth == 0:
                ops.append(cur.strip())
                cur = ""
            else:
                cur += ch
        if cur.strip():
            ops.append(cur.strip())
        return ops

    def is_xmm(self, o):
        return o.startswith("%xmm")

    def xmm(self, o):
        return "x" + o[4:]

    def is_gpr(self, o):
        return o.startswith("%") and o[1:] in ALIAS

    def mem_ref(self, o, comment, size=8):
        """Return a C lvalue/rvalue expression for a memory operand."""
        if "(%rip)" in o:
            m = re.search(r"0x([0-9a-f]+)\s*$", comment)
            addr = int(m.group(1), 16)
            base = None
            for tb, sz in TABLES.items():
                if tb <= addr < tb + sz:
                    base = tb
            if base is not None:
                self.used_tables.add(base)
                return "T_%x[%d]" % (base, (addr - base) // 8), "u"
            self.consts[addr] = rodata_u64(addr)
            return "K_%x" % addr, "u"
        if o.startswith("%fs:"):
            return None, "fs"
        m = re.match(r"(-?0x[0-9a-f]+|-?\d+)?\((%\w+)(?:,(%\w+),(\d+))?\)$", o)
        assert m, o
        disp = int(m.group(1), 0) if m.group(1) else 0
        base = m.group(2)[1:]
        if base == "rsp":
            return "S_%s" % (("m%x" % -disp) if disp < 0 else ("%x" % disp)), "stack"
        assert base in self.ptrbase, (self.name, o, self.ptrbase)
        tb = self.ptrbase[base]
        self.used_tables.add(tb)
        idx = ""
        if m.group(3):
            idx = " + %s * %s" % (self.gpr_read(m.group(3)[1:]), m.group(4))
        expr = "(%s - 0x%xull + %d%s)" % (base, tb, disp, idx)
        return "T_%x[%s / 8]" % (tb, expr), "u"

    def gpr_read(self, r):
        reg, w = ALIAS[r]
        if w == 64:
            return reg
        if w == 32:
            return "((uint32_t)%s)" % reg
        if w == 8:
            return "((uint8_t)%s)" % reg
        return "((uint8_t)(%s >> 8))" % reg

    def gpr_write(self, r, expr):
        reg, w = ALIAS[r]
        self.ptrbase.pop(reg, None)
        if w == 64:
            return "%s = (uint64_t)(%s);" % (reg, expr)
        if w == 32:
            return "%s = (uint64_t)(uint32_t)(%s);" % (reg, expr)
        if w == 8:
            return "%s = (%s & ~0xffull) | (uint64_t)(uint8_t)(%s);" % (reg, reg, expr)
        return "%s = (%s & ~0xff00ull) | ((uint64_t)(uint8_t)(%s) << 8);" % (reg, reg, expr)

    def imm(self, o):
        v = int(o[1:], 0)
        return v

    def fval(self, o, comment):
        """double-valued source operand."""
        if self.is_xmm(o):
            return "%s.d" % self.xmm(o)
        ref, kind = self.mem_ref(o, comment)
        if kind == "stack":
            return "%s.d" % ref
        return "hm_u2d(%s)" % ref

    def uval(self, o, comment):
        """64-bit pattern source operand."""
        if self.is_xmm(o):
            return "%s.u" % self.xmm(o)
        if self.is_gpr(o):
            return self.gpr_read(o[1:])
        if o.startswith("$"):
            return "0x%xull" % (self.imm(o) & 0xFFFFFFFFFFFFFFFF)
        ref, kind = self.mem_ref(o, comment)
        if kind == "stack":
            return "%s.u" % ref
        if kind == "fs":
            return "0ull"
        return ref

    # ---- translation -----------------------------------------------------
    def cond(self, mn):
        f = self.flags
        assert f is not None, (self.name, mn)
        kind = f[0]
        if kind == "fcmp":      # comisd: a = op2 compared with b = op1
            a, b = f[1], f[2]
            return {"ja": "(%s > %s)" % (a, b), "jae": "(%s >= %s)" % (a, b),
                    "jb": "(!(%s >= %s))" % (a, b), "jbe": "(!(%s > %s))" % (a, b),
                    "je": "(!(%s < %s || %s > %s))" % (a, b, a, b),
                    "jne": "(%s < %s || %s > %s)" % (a, b, a, b),
                    "jp": "(%s != %s || %s != %s)" % (a, a, b, b)}[mn]
        if kind == "icmp":      # cmp b, a  -> flags of a - b, width w
            a, b, w = f[1], f[2], f[3]
            st = {32: "int32_t", 64: "int64_t", 8: "int8_t"}[w]
            ut = {32: "uint32_t", 64: "uint64_t", 8: "uint8_t"}[w]
            sa, sb = "(%s)(%s)" % (st, a), "(%s)(%s)" % (st, b)
            ua, ub = "(%s)(%s)" % (ut, a), "(%s)(%s)" % (ut, b)
            return {"je": "(%s == %s)" % (ua, ub), "jne": "(%s != %s)" % (ua, ub),
                    "jg": "(%s > %s)" % (sa, sb), "jle": "(%s <= %s)" % (sa, sb),
                    "jge": "(%s >= %s)" % (sa, sb), "jl": "(%s < %s)" % (sa, sb),
                    "ja": "(%s > %s)" % (ua, ub), "jbe": "(%s <= %s)" % (ua, ub),
                    "jae": "(%s >= %s)" % (ua, ub), "jb": "(%s < %s)" % (ua, ub)}[mn]
        if kind == "test":      # result r of width w
            r, w = f[1], f[2]
            st = {32: "int32_t", 64: "int64_t", 8: "int8_t"}[w]
            ut = {32: "uint32_t", 64: "uint64_t", 8: "uint8_t"}[w]
            return {"je": "((%s)(%s) == 0)" % (ut, r), "jne": "((%s)(%s) != 0)" % (ut, r),
                    "js": "((%s)(%s) < 0)" % (st, r), "jns": "((%s)(%s) >= 0)" % (st, r),
                    "jle": "((%s)(%s) <= 0)" % (st, r), "jg": "((%s)(%s) > 0)" % (st, r)}[mn]
        raise AssertionError(f)

    def emit(self, s):
        self.out.append("    " + s)

    def translate(self):
        e = self.emit
        for (addr, mn, ops_s, comment) in self.lines:
            if addr in self.targets:
                self.out.append("L_%x:" % addr)
            ops = self.split_ops(ops_s)
            if mn in ("endbr64", "nop", "nopl", "nopw", "pushq", "popq", "file"):
                continue
            if mn == "retq":
                e("return x0.d;")
                self.flags = None
                continue
            if mn in ("vstmxcsr",):
                ref, _ = self.mem_ref(ops[0], comment)
                e("%s.u = 0x1f80ull;  /* default MXCSR: round-to-nearest */" % ref)
                continue
            if mn in ("vldmxcsr",):
                e("/* vldmxcsr: rounding mode unchanged (nearest) */")
                continue
            if mn == "jmp":
                t = int(ops[0].split()[0], 16)
                if t in EXTERN:
                    self.extern(EXTERN[t])
                else:
                    e("goto L_%x;" % t)
                continue
            if mn.startswith("j"):
                t = int(ops[0].split()[0], 16)
                c = self.cond(mn)
                if t in EXTERN:
                    e("if %s { %s }" % (c, self.extern_str(EXTERN[t])))
                else:
                    e("if %s goto L_%x;" % (c, t))
                continue
            if mn == "callq":
                t = int(ops[0].split()[0], 16)
                self.extern(EXTERN[t])
                continue
            # ---- moves ----
            if mn in ("vmovsd", "vmovq"):
                if len(ops) == 3:   # vmovsd %xa, %xb, %xc : low from xa
                    e("%s.u = %s.u;" % (self.xmm(ops[2]), self.xmm(ops[0])))
                    continue
                src, dst = ops
                if self.is_xmm(dst):
                    if self.is_gpr(src):
                        e("%s.u = %s;" % (self.xmm(dst), self.gpr_read(src[1:])))
                    else:
                        e("%s.u = %s;" % (self.xmm(dst), self.uval(src, comment)))
                elif self.is_gpr(dst):
                    e(self.gpr_write(dst[1:], self.uval(src, comment)))
                else:
                    ref, kind = self.mem_ref(dst, comment)
                    assert kind == "stack"
                    e("%s.u = %s;" % (ref, self.uval(src, comment)))
                continue
            if mn in ("movq", "movl", "movabsq"):
                src, dst = ops
                if dst.startswith("%fs:"):
                    continue
                if self.is_gpr(dst):
                    if src.startswith("$"):
                        v = self.imm(src) & 0xFFFFFFFFFFFFFFFF
                        e(self.gpr_write(dst[1:], "0x%xull" % v))
                    elif "(%rip)" in src and ("0xe5f" in comment or "0xe60" in comment):
                        e(self.gpr_write(dst[1:], "0ull") + "  /* GOT (errno/cpu features) */")
                    else:
                        val = self.uval(src, comment)
                        e(self.gpr_write(dst[1:], val))
                        if self.is_gpr(src) and ALIAS[src[1:]][0] in self.ptrbase:
                            self.ptrbase[ALIAS[dst[1:]][0]] = self.ptrbase[ALIAS[src[1:]][0]]
                else:
                    ref, kind = self.mem_ref(dst, comment)
                    if kind == "fs":
                        continue
                    assert kind == "stack"
                    if src.startswith("$"):
                        e("%s.u = 0x%xull;" % (ref, self.imm(src) & 0xFFFFFFFFFFFFFFFF))
                    else:
                        w = 32 if mn == "movl" else 64
                        val = self.uval(src, comment)
                        if w == 32:
                            e("%s.u = (%s.u & ~0xffffffffull) | (uint32_t)(%s);" % (ref, ref, val))
                        else:
                            e("%s.u = %s;" % (ref, val))
                continue
            if mn == "leaq":
                src, dst = ops
                if "(%rip)" in src:
                    m = re.search(r"0x([0-9a-f]+)", comment)
                    a = int(m.group(1), 16)
                    reg = ALIAS[dst[1:]][0]
                    e("%s = 0x%xull;" % (reg, a))
                    assert a in TABLES, hex(a)
                    self.ptrbase[reg] = a
                else:
                    e("/* %s %s (address of stack slot, only for __branred) */" % (mn, ops_s))
                    ref, kind = self.mem_ref(src, comment)
                    assert kind == "stack", (self.name, ops_s)
                    self.lea_stack[ALIAS[dst[1:]][0]] = ref
                continue
            if mn == "leal":
                src, dst = ops
                m = re.match(r"(-?0x[0-9a-f]+|-?\d+)?\((%\w+)\)$", src)
                disp = int(m.group(1), 0) if m.group(1) else 0
                e(self.gpr_write(dst[1:], "%s + (uint64_t)(%d)" % (self.gpr_read(m.group(2)[1:]), disp)))
                continue
            if mn in ("movslq", "cltq"):
                if mn == "cltq":
                    e("rax = (uint64_t)(int64_t)(int32_t)(uint32_t)rax;")
                else:
                    src, dst = ops
                    keep = ALIAS[src[1:]][0] in self.ptrbase
                    e(self.gpr_write(dst[1:], "(uint64_t)(int64_t)(int32_t)%s" % self.gpr_read(src[1:])))
                continue
            # ---- integer ALU ----
            if mn in ("addq", "subq", "andq", "addl", "andl", "orl", "xorl", "andb",
                      "shll", "shlq", "shrq", "sarq"):
                src, dst = ops
                if dst == "%rsp":
                    continue
                w = {"q": 64, "l": 32, "b": 8}[mn[-1]]
                if ALIAS[dst[1:]][1] == "h":
                    w = 8
                d = self.gpr_read(dst[1:])
                s = self.uval(src, comment)
                op = mn[:-1]
                if op == "xor" and src == dst:
                    e(self.gpr_write(dst[1:], "0"))
                    self.flags = ("test", "0", w)
                    continue
                dreg = ALIAS[dst[1:]][0]
                pb = self.ptrbase.get(dreg)
                if pb is None and op == "add" and self.is_gpr(src):
                    pb = self.ptrbase.get(ALIAS[src[1:]][0])
                if op in ("add", "sub", "and", "or", "xor"):
                    cop = {"add": "+", "sub": "-", "and": "&", "or": "|", "xor": "^"}[op]
                    r = "(%s %s %s)" % (d, cop, s)
                elif op == "shl":
                    r = "(%s << %s)" % (d, s)
                elif op == "shr":
                    r = "(%s >> %s)" % (d, s)
                elif op == "sar":
                    r = "(uint64_t)((int64_t)%s >> %s)" % (d, s)
                if w == 32:
                    r = "(uint32_t)" + r
                e(self.gpr_write(dst[1:], r))
                if op == "add" and pb is not None:
                    self.ptrbase[dreg] = pb
                if op == "sub" and "%fs:" in src:
                    self.flags = ("test", d, w)
                else:
                    self.flags = ("test", self.gpr_read(dst[1:]), w)
                continue
            if mn in ("cmpl", "cmpq"):
                src, dst = ops
                w = 32 if mn == "cmpl" else 64
                self.flags = ("icmp", self.uval(dst, comment), self.uval(src, comment), w)
                continue
            if mn in ("testl", "testb"):
                a, b = ops
                w = 32 if mn == "testl" else 8
                self.flags = ("test", "(%s & %s)" % (self.uval(a, comment), self.uval(b, comment)), w)
                continue
            # ---- float ----
            if mn in ("vaddsd", "vsubsd", "vmulsd", "vdivsd"):
                s1, s2, dst = ops
                op = {"vaddsd": "+", "vsubsd": "-", "vmulsd": "*", "vdivsd": "/"}[mn]
                e("%s.d = %s %s %s;" % (self.xmm(dst), self.fval(s2, comment), op, self.fval(s1, comment)))
                continue
            m = re.match(r"v(fn?m(?:add|sub))(132|213|231)sd", mn)
            if m:
                kind, order = m.group(1), m.group(2)
                s1, s2, dst = ops
                D, A, B = "%s.d" % self.xmm(dst), self.fval(s1, comment), self.fval(s2, comment)
                if order == "132":
                    p, q, c = D, A, B
                elif order == "213":
                    p, q, c = B, D, A
                else:
                    p, q, c = B, A, D
                neg = kind.startswith("fn")
                sub = kind.endswith("sub")
                e("%s.d = fma(%s%s, %s, %s%s);" % (self.xmm(dst), "-" if neg else "", p, q,
                                                  "-" if sub else "", c))
                continue
            if mn in ("vandpd", "vorpd", "vxorpd", "vxorps"):
                s1, s2, dst = ops
                op = {"vandpd": "&", "vorpd": "|", "vxorpd": "^", "vxorps": "^"}[mn]
                if s1 == s2 and op == "^":
                    e("%s.u = 0;" % self.xmm(dst))
                else:
                    e("%s.u = %s %s %s;" % (self.xmm(dst), self.uval(s2, comment), op, self.uval(s1, comment)))
                continue
            if mn in ("vcomisd", "ucomisd", "vucomisd"):
                s1, s2 = ops
                self.flags = ("fcmp", self.fval(s2, comment), self.fval(s1, comment))
                continue
            if mn in ("vcmpltsd", "vcmpnltsd"):
                s1, s2, dst = ops
                c = "(%s < %s)" % (self.fval(s2, comment), self.fval(s1, comment))
                if mn == "vcmpnltsd":
                    c = "(!%s)" % c
                e("%s.u = %s ? ~0ull : 0ull;" % (self.xmm(dst), c))
                continue
            if mn == "vblendvpd":
                mk, a, b, dst = ops
                e("%s.u = (%s.u >> 63) ? %s : %s;" % (self.xmm(dst), self.xmm(mk),
                                                      self.uval(a, comment), self.uval(b, comment)))
                continue
            if mn == "vcvtsi2sd":
                src, _, dst = ops
                e("%s.d = (double)(int32_t)%s;" % (self.xmm(dst), self.gpr_read(src[1:])))
                continue
            if mn == "vcvttsd2si":
                src, dst = ops
                e(self.gpr_write(dst[1:], "(uint32_t)(int32_t)%s.d" % self.xmm(src)))
                continue
            raise NotImplementedError((self.name, hex(addr), mn, ops_s))

    def extern_str(self, what):
        if what == "branred":
            # int __branred(double x, double *a, double *aa): x in xmm0, a/aa
            # the stack slots the preceding leaq's put in rdi/rsi (hm_branred.h)
            a, aa = self.lea_stack["rdi"], self.lea_stack["rsi"]
            return ("{ double ba_ = 0.0, baa_ = 0.0; rax = (uint64_t)(uint32_t)hm_branred(x0.d, &ba_, &baa_); "
                    "%s.d = ba_; %s.d = baa_; }" % (a, aa))
        if what == "math_invalid":
            return "*unsupported = 2; return (x0.d - x0.d) / (x0.d - x0.d);"
        if what == "math_divzero":
            return "*unsupported = 2; return -HUGE_VAL;"
        if what == "stack_chk_fail":
            return "*unsupported = 3; return 0.0;"
        raise AssertionError(what)

    def extern(self, what):
        self.emit(self.extern_str(what))

    def render(self):
        self.translate()
        xs = sorted({int(x) for x in re.findall(r"\bx(\d+)\.", "\n".join(self.out))} | {0})
        S = sorted(set(re.findall(r"\bS_(m?[0-9a-f]+)\.", "\n".join(self.out))))
        hdr = ["HM_EMUL_FN double hm_glibc_%s(double arg, int* unsupported)" % self.name, "{"]
        hdr.append("    uint64_t rax = 0, rbx = 0, rcx = 0, rdx = 0, rsi = 0, rdi = 0, rbp = 0;")
        hdr.append("    hm_x64 %s;" % ", ".join("x%d" % i for i in xs))
        if S:
            hdr.append("    hm_x64 %s;" % ", ".join("S_%s" % s for s in S))
            for s in S:
                hdr.append("    S_%s.u = 0;" % s)
        for i in xs:
            hdr.append("    x%d.u = 0;" % i)
        hdr.append("    x0.d = arg;")
        hdr.append("    (void)rax; (void)rbx; (void)rcx; (void)rdx; (void)rsi; (void)rdi; (void)rbp;")
        body = self.out
        return "\n".join(hdr + body + ["}"])


def main():
    parts = []
    consts = {}
    tables = set()
    for name, a, b in FUNCS:
        t = Tr(name, a, b)
        parts.append(t.render())
        consts.update(t.consts)
        tables |= t.used_tables
    o = []
    o.append("/* GENERATED by tools/glibc_emul/gen_glibc_emul.py -- do not edit.")
    o.append(" * Bit-exact restatement of glibc 2.35 libm (Ubuntu 2.35-0ubuntu3.11) __tan_fma,")
    o.append(" * __cos_fma and __log_fma for the device slow path.  Operation order and FMA")
    o.append(" * contractions follow the library's machine code one instruction at a time;")
    o.append(" * constants and tables are the library's .rodata words.  glibc is LGPL-2.1;")
    o.append(" * this file restates its arithmetic so tile rows match CPython's math module")
    o.append(" * (reference tile.py:17) bit for bit.  Checked against the live libm by")
    o.append(" * tests/test_math_host.py::test_glibc_restatement_bit_exact. */")
    o.append("#pragma once")
    o.append('#include "hm_common.h"')
    o.append('#include "hm_branred.h"')
    o.append("")
    o.append("HM_EMUL_BEGIN")
    o.append("")
    for a in sorted(consts):
        u = consts[a]
        o.append("#define K_%x 0x%016xull" % (a, u))
    o.append("")
    for tb in sorted(tables):
        n = TABLES[tb] // 8
        vals = [rodata_u64(tb + 8 * i) for i in range(n)]
        o.append("HM_EMUL_TABLE uint64_t T_%x[%d] = {" % (tb, n))
        for i in range(0, n, 4):
            o.append("    " + ", ".join("0x%016xull" % v for v in vals[i:i + 4]) + ",")
        o.append("};")
        o.append("")
    o.extend(parts)
    o.append("")
    o.append("HM_EMUL_END")
    print("\n".join(o))


if __name__ == "__main__":
    main()
