"""Condensed view of a kernel's MFMA loop blocks in a gfx950 .s file (dev tool).
usage: python tools/isa_loop.py file.s mangled_kernel_name [max_blocks]"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    nmax = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    s = open(path).read()
    start = s.index(name + ':')
    end = s.index('.Lfunc_end', start)
    body = s[start:end].split('\n')
    labels = [(i, l) for i, l in enumerate(body) if re.match(r'^\.LBB\d+_\d+:', l)]
    shown = 0
    for k, (i, l) in enumerate(labels):
        j = labels[k + 1][0] if k + 1 < len(labels) else len(body)
        seg = body[i:j]
        cnt = lambda p: sum(1 for x in seg if re.search(p, x))  # noqa: E731
        if cnt('v_mfma') == 0:
            continue
        print(l[:14], j - i, 'mfma', cnt('v_mfma'), 'ds_read', cnt('ds_read'), 'wait', cnt('s_waitcnt'),
              'dma', cnt('lds_dword|offen lds'), 'bar', cnt('s_barrier'), 'scratch', cnt('scratch_'))
        if shown >= nmax:
            continue
        shown += 1
        out = []
        for x in seg:
            x = x.strip()
            if not x or x.startswith(';'):
                continue
            t = x.split()[0]
            tag = 'MFMA' if t.startswith('v_mfma') else (
                'VALU' if re.match(r'v_(add|sub|subrev)_f32', t) else None)
            if tag:
                if out and out[-1].startswith(tag + 'x'):
                    out[-1] = f'{tag}x{int(out[-1][len(tag) + 1:]) + 1}'
                else:
                    out.append(f'{tag}x1')
            elif t.startswith(('ds_', 's_waitcnt', 's_barrier', 'buffer_', 'global_', 's_sched', 's_nop')):
                out.append(x.split(';')[0][:48])
        print('  ' + ' | '.join(out))


if __name__ == '__main__':
    main()
