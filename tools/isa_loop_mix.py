"""Instruction mix of a kernel's main loop in a gfx950 disassembly (tools/isa_dump.sh output): the backward branch
whose body holds the most MFMAs, its instructions counted by class and the most frequent VALU opcodes.
    python tools/isa_loop_mix.py DUMP.s KERNEL_SUBSTRING [KERNEL_SUBSTRING ...]"""
import re
import sys
from collections import Counter


def loop_mix(txt: str, want: str):
    funcs = re.split(r'\n(?=[0-9a-f]+ <[^>]+>:\n)', txt)
    for f in funcs:
        m = re.match(r'[0-9a-f]+ <([^>]+)>:', f)
        if not m or want not in m.group(1):
            continue
        lines = f.split('\n')
        addr = {}
        for i, l in enumerate(lines):
            mm = re.search(r'//\s*([0-9A-F]+):', l)
            if mm:
                addr[int(mm.group(1), 16)] = i
        best = None
        for i, l in enumerate(lines):
            mm = re.match(r'\s*s_cbranch_\w+\s+(\d+)', l.split('//')[0])
            if not mm:
                continue
            off = int(mm.group(1))
            off = off - 65536 if off >= 32768 else off
            if off >= 0:
                continue
            pc = int(re.search(r'//\s*([0-9A-F]+):', l).group(1), 16)
            j = addr.get(pc + 4 + 4 * off)
            if j is None:
                continue
            body = lines[j:i + 1]
            nm = sum('v_mfma' in b for b in body)
            if nm and (best is None or nm > best[0]):
                best = (nm, body)
        if best is None:
            continue
        ops = [b.split('//')[0].strip().split(' ')[0] for b in best[1]]
        ops = [o for o in ops if o]
        cls = Counter('mfma' if o.startswith('v_mfma') else 'valu' if o.startswith('v_') else
                      'salu' if o.startswith('s_') else o.split('_')[0] for o in ops)
        valu = Counter(o for o in ops if o.startswith('v_') and not o.startswith('v_mfma'))
        yield m.group(1), len(ops), dict(cls), valu.most_common(12)


if __name__ == "__main__":
    txt = open(sys.argv[1]).read()
    for w in sys.argv[2:]:
        for name, n, cls, valu in loop_mix(txt, w):
            print(name[-60:], n, cls)
            print("   ", valu)


def skeleton(txt: str, want: str, limit: int = 60):
    """Branches, barriers, LDS-DMA / vector-memory issues and vmcnt waits of a kernel, MFMA runs collapsed."""
    funcs = re.split(r'\n(?=[0-9a-f]+ <[^>]+>:\n)', txt)
    for f in funcs:
        m = re.match(r'[0-9a-f]+ <([^>]+)>:', f)
        if not m or want not in m.group(1):
            continue
        out, run = [], 0
        for i, l in enumerate(f.split('\n')):
            op = l.split('//')[0].strip()
            if op.startswith('v_mfma'):
                run += 1
                continue
            if re.match(r'(s_cbranch|s_barrier|global_load|buffer_load|s_waitcnt.*vmcnt)', op):
                if run:
                    out.append(f'      mfma x{run}')
                    run = 0
                out.append(f'{i:5d}: {op}')
        if run:
            out.append(f'      mfma x{run}')
        print(m.group(1)[-60:])
        print('\n'.join(out[:limit]))
