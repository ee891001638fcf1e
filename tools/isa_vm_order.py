"""ISA audit of counted-vmcnt pipelines: for one kernel of a disassembled gfx950 code object, print the sequence of
vector-memory issues (LDS-DMA `buffer_load ... lds`, register `global_load` / `buffer_load`, stores), `s_waitcnt
vmcnt(N)` waits, barriers and branches, so the issue order each counted wait assumes can be read off.

usage: python tools/isa_vm_order.py DIS.s KERNEL_SUBSTRING [--all]
(DIS.s: llvm-objdump -d --mcpu=gfx950 of the unbundled code object; see tools/isa_dump.sh)"""
import re
import sys


def kernel_lines(path, name):
    out, on = [], False
    for line in open(path):
        if re.match(r"^[0-9a-f]+ <", line):
            on = name in line
            if on:
                out.append(line.rstrip())
            continue
        if on:
            out.append(line.rstrip())
    return out


def main():
    path, name = sys.argv[1], sys.argv[2]
    for line in kernel_lines(path, name):
        ins = line.split("//")[0].strip()
        if not ins:
            continue
        tag = None
        if re.match(r"(buffer|global)_load\S*", ins) and " lds" in ins:
            tag = "DMA "
        elif re.match(r"(buffer|global)_load", ins):
            tag = "LOAD"
        elif re.match(r"(buffer|global)_store", ins):
            tag = "STOR"
        elif ins.startswith("s_waitcnt") and "vmcnt" in ins:
            tag = "WAIT"
        elif ins.startswith("s_barrier"):
            tag = "BAR "
        elif re.match(r"s_(cbranch|branch)", ins):
            tag = "BR  "
        elif ins.startswith("<") or line.startswith("0"):
            tag = "----"
        if tag:
            print(tag, ins[:110])


if __name__ == "__main__":
    main()
