#!/usr/bin/env python3
"""Read-only JVM class-file disassembler (static reading of the MHAP jar's bytecode).

canu runs MHAP as a prebuilt jar (src/mhap/mhap-2.1.2.tar, OverlapMhap.pm:374-498); no Java
sources or fixtures ship with it and no JVM exists here, so the jar is never run.  This tool
parses class files as DATA -- constant pool, methods, bytecode -- and prints a method's
instructions with their constants resolved, so that oracle/mhap_jar.py's restatement
(hash family, seeding, weighting) can be checked against what the bytecode does.

    python tools/classfile.py edu/umd/marbl/mhap/sketch/HashUtils [method-substring]
"""
from __future__ import annotations

import io
import os
import struct
import sys
import tarfile
import zipfile

JAR_TAR = "/root/reference/src/mhap/mhap-2.1.2.tar"

# opcode -> (mnemonic, operand format): b/B s1/u1, h/H s2/u2, i s4; special: tableswitch,
# lookupswitch, wide
_OPS = {}


def _op(code, name, fmt=""):
    _OPS[code] = (name, fmt)


for i, n in enumerate(["nop", "aconst_null", "iconst_m1", "iconst_0", "iconst_1", "iconst_2",
                       "iconst_3", "iconst_4", "iconst_5", "lconst_0", "lconst_1", "fconst_0",
                       "fconst_1", "fconst_2", "dconst_0", "dconst_1"]):
    _op(i, n)
_op(0x10, "bipush", "b"); _op(0x11, "sipush", "h"); _op(0x12, "ldc", "B")
_op(0x13, "ldc_w", "H"); _op(0x14, "ldc2_w", "H")
for i, n in enumerate(["iload", "lload", "fload", "dload", "aload"]):
    _op(0x15 + i, n, "B")
for t, base in (("i", 0x1a), ("l", 0x1e), ("f", 0x22), ("d", 0x26), ("a", 0x2a)):
    for j in range(4):
        _op(base + j, f"{t}load_{j}")
for i, n in enumerate(["iaload", "laload", "faload", "daload", "aaload", "baload", "caload",
                       "saload"]):
    _op(0x2e + i, n)
for i, n in enumerate(["istore", "lstore", "fstore", "dstore", "astore"]):
    _op(0x36 + i, n, "B")
for t, base in (("i", 0x3b), ("l", 0x3f), ("f", 0x43), ("d", 0x47), ("a", 0x4b)):
    for j in range(4):
        _op(base + j, f"{t}store_{j}")
for i, n in enumerate(["iastore", "lastore", "fastore", "dastore", "aastore", "bastore",
                       "castore", "sastore", "pop", "pop2", "dup", "dup_x1", "dup_x2", "dup2",
                       "dup2_x1", "dup2_x2", "swap"]):
    _op(0x4f + i, n)
_arith = []
for op in ("add", "sub", "mul", "div", "rem", "neg"):
    for t in "ilfd":
        _arith.append(t + op)
for i, n in enumerate(_arith):
    _op(0x60 + i, n)
for i, n in enumerate(["ishl", "lshl", "ishr", "lshr", "iushr", "lushr", "iand", "land", "ior",
                       "lor", "ixor", "lxor"]):
    _op(0x78 + i, n)
_op(0x84, "iinc", "Bb")
for i, n in enumerate(["i2l", "i2f", "i2d", "l2i", "l2f", "l2d", "f2i", "f2l", "f2d", "d2i",
                       "d2l", "d2f", "i2b", "i2c", "i2s", "lcmp", "fcmpl", "fcmpg", "dcmpl",
                       "dcmpg"]):
    _op(0x85 + i, n)
for i, n in enumerate(["ifeq", "ifne", "iflt", "ifge", "ifgt", "ifle", "if_icmpeq", "if_icmpne",
                       "if_icmplt", "if_icmpge", "if_icmpgt", "if_icmple", "if_acmpeq",
                       "if_acmpne", "goto", "jsr"]):
    _op(0x99 + i, n, "j")
_op(0xa9, "ret", "B"); _op(0xaa, "tableswitch", "T"); _op(0xab, "lookupswitch", "L")
for i, n in enumerate(["ireturn", "lreturn", "freturn", "dreturn", "areturn", "return"]):
    _op(0xac + i, n)
for i, n in enumerate(["getstatic", "putstatic", "getfield", "putfield", "invokevirtual",
                       "invokespecial", "invokestatic"]):
    _op(0xb2 + i, n, "H")
_op(0xb9, "invokeinterface", "HBB"); _op(0xba, "invokedynamic", "HBB"); _op(0xbb, "new", "H")
_op(0xbc, "newarray", "B"); _op(0xbd, "anewarray", "H"); _op(0xbe, "arraylength")
_op(0xbf, "athrow"); _op(0xc0, "checkcast", "H"); _op(0xc1, "instanceof", "H")
_op(0xc2, "monitorenter"); _op(0xc3, "monitorexit"); _op(0xc4, "wide", "W")
_op(0xc5, "multianewarray", "HB"); _op(0xc6, "ifnull", "j"); _op(0xc7, "ifnonnull", "j")
_op(0xc8, "goto_w", "J"); _op(0xc9, "jsr_w", "J")


class ClassFile:
    def __init__(self, data: bytes):
        self.d = data
        self.p = 8
        n = self._u2()
        self.cp = [None] * n
        i = 1
        while i < n:
            tag = self._u1()
            if tag == 1:
                ln = self._u2()
                self.cp[i] = ("utf8", self.d[self.p:self.p + ln].decode("utf-8", "replace"))
                self.p += ln
            elif tag in (3, 4):
                raw = self.d[self.p:self.p + 4]
                self.p += 4
                self.cp[i] = ("int", struct.unpack(">i", raw)[0]) if tag == 3 else \
                    ("float", struct.unpack(">f", raw)[0])
            elif tag in (5, 6):
                raw = self.d[self.p:self.p + 8]
                self.p += 8
                self.cp[i] = ("long", struct.unpack(">q", raw)[0]) if tag == 5 else \
                    ("double", struct.unpack(">d", raw)[0])
                i += 1
            elif tag in (7, 8, 16, 19, 20):
                self.cp[i] = ({7: "class", 8: "string", 16: "mtype", 19: "module",
                               20: "package"}[tag], self._u2())
            elif tag in (9, 10, 11, 12, 17, 18):
                self.cp[i] = ({9: "field", 10: "method", 11: "imethod", 12: "nat", 17: "dyn",
                               18: "indy"}[tag], self._u2(), self._u2())
            elif tag == 15:
                self.cp[i] = ("mhandle", self._u1(), self._u2())
            else:
                raise ValueError(f"constant pool tag {tag}")
            i += 1
        self.access, self.this, self.super = self._u2(), self._u2(), self._u2()
        n_if = self._u2()
        self.p += 2 * n_if
        self.fields = [self._member() for _ in range(self._u2())]
        self.methods = [self._member() for _ in range(self._u2())]

    def _u1(self):
        v = self.d[self.p]
        self.p += 1
        return v

    def _u2(self):
        v = struct.unpack(">H", self.d[self.p:self.p + 2])[0]
        self.p += 2
        return v

    def _u4(self):
        v = struct.unpack(">I", self.d[self.p:self.p + 4])[0]
        self.p += 4
        return v

    def _member(self):
        acc, name, desc = self._u2(), self._u2(), self._u2()
        attrs = {}
        for _ in range(self._u2()):
            an, ln = self._u2(), self._u4()
            attrs[self.utf(an)] = self.d[self.p:self.p + ln]
            self.p += ln
        return {"access": acc, "name": self.utf(name), "desc": self.utf(desc), "attrs": attrs}

    def utf(self, i):
        return self.cp[i][1]

    def const(self, i) -> str:
        e = self.cp[i]
        k = e[0]
        if k == "utf8":
            return repr(e[1])
        if k in ("int", "long", "float", "double"):
            return f"{e[1]!r}" + (f" (0x{e[1] & 0xFFFFFFFFFFFFFFFF:x})" if k == "long" else "")
        if k == "class":
            return self.utf(e[1])
        if k == "string":
            return repr(self.utf(e[1]))
        if k == "nat":
            return f"{self.utf(e[1])}:{self.utf(e[2])}"
        if k in ("field", "method", "imethod"):
            return f"{self.const(e[1])}.{self.const(e[2])}"
        if k == "indy":
            return f"indy#{e[1]} {self.const(e[2])}"
        return str(e)

    def disassemble(self, m) -> list[str]:
        code = m["attrs"].get("Code")
        if code is None:
            return ["  (no code)"]
        max_stack, max_locals, ln = struct.unpack(">HHI", code[:8])
        bc = code[8:8 + ln]
        out = [f"  max_stack {max_stack} max_locals {max_locals} code {ln} B"]
        pc = 0
        while pc < ln:
            op = bc[pc]
            name, fmt = _OPS.get(op, (f"op_{op:02x}", ""))
            q = pc + 1
            args = []
            if fmt == "T":
                q = (q + 3) & ~3
                dflt, lo, hi = struct.unpack(">iii", bc[q:q + 12])
                q += 12
                tgts = struct.unpack(f">{hi - lo + 1}i", bc[q:q + 4 * (hi - lo + 1)])
                q += 4 * (hi - lo + 1)
                args.append(f"[{lo}..{hi}] -> {[pc + t for t in tgts]} default {pc + dflt}")
            elif fmt == "L":
                q = (q + 3) & ~3
                dflt, npairs = struct.unpack(">ii", bc[q:q + 8])
                q += 8
                pairs = [struct.unpack(">ii", bc[q + 8 * k:q + 8 * k + 8]) for k in range(npairs)]
                q += 8 * npairs
                args.append(f"{[(a, pc + b) for a, b in pairs]} default {pc + dflt}")
            elif fmt == "W":
                op2 = bc[q]
                name = "wide " + _OPS[op2][0]
                q += 1
                if op2 == 0x84:
                    args += [str(struct.unpack(">H", bc[q:q + 2])[0]),
                             str(struct.unpack(">h", bc[q + 2:q + 4])[0])]
                    q += 4
                else:
                    args.append(str(struct.unpack(">H", bc[q:q + 2])[0]))
                    q += 2
            else:
                for f in fmt:
                    if f == "b":
                        args.append(str(struct.unpack(">b", bc[q:q + 1])[0])); q += 1
                    elif f == "B":
                        v = bc[q]; q += 1
                        args.append(self.const(v) if name == "ldc" else str(v))
                    elif f == "h":
                        args.append(str(struct.unpack(">h", bc[q:q + 2])[0])); q += 2
                    elif f == "H":
                        v = struct.unpack(">H", bc[q:q + 2])[0]; q += 2
                        args.append(self.const(v) if name not in ("iinc",) else str(v))
                    elif f == "j":
                        args.append(f"-> {pc + struct.unpack('>h', bc[q:q + 2])[0]}"); q += 2
                    elif f == "J":
                        args.append(f"-> {pc + struct.unpack('>i', bc[q:q + 4])[0]}"); q += 4
            out.append(f"  {pc:5d}: {name} {' '.join(args)}".rstrip())
            pc = q
        return out


def load(cls: str, jar_tar: str = JAR_TAR) -> ClassFile:
    with tarfile.open(jar_tar) as t:
        jar = [m for m in t.getmembers() if m.name.endswith(".jar")][0]
        data = t.extractfile(jar).read()
    with zipfile.ZipFile(io.BytesIO(data)) as z:
        return ClassFile(z.read(cls + ".class"))


def main():
    if len(sys.argv) < 2:
        print(__doc__)
        return
    cf = load(sys.argv[1])
    pick = sys.argv[2] if len(sys.argv) > 2 else None
    for m in cf.methods:
        if pick is not None and pick not in m["name"]:      # "" disassembles every method
            continue
        print(f"{m['name']}{m['desc']}")
        if pick is not None:
            print("\n".join(cf.disassemble(m)))


if __name__ == "__main__":
    main()
