"""Resolve preprocessor conditionals on given macros (a small unifdef):
    python scripts/dbg/unifdef.py FILE NAME=VALUE ...
Removes '#ifndef NAME / #define NAME v / #endif' default blocks of the named macros,
evaluates '#if' / '#elif' lines whose expression uses only named macros (and literals),
keeps the taken branch, and substitutes the names by their values in the remaining
code.  Conditionals on other macros are left alone."""
import re
import sys


def cexpr(e, vals):
    e = re.sub(r'//.*', '', e)
    e = re.sub(r'defined\((\w+)\)', lambda m: '1' if m.group(1) in vals else '0', e)
    for k, v in vals.items():
        e = re.sub(r'\b%s\b' % k, str(v), e)
    if re.search(r'[A-Za-z_]', e.replace('and', '').replace('or', '').replace('not', '')):
        return None
    e = e.replace('&&', ' and ').replace('||', ' or ')
    e = re.sub(r'!(?!=)', ' not ', e)
    return int(bool(eval(e)))


def main():
    path = sys.argv[1]
    vals = dict(a.split('=') for a in sys.argv[2:])
    vals = {k: int(v) for k, v in vals.items()}
    lines = open(path).read().split('\n')
    out = []
    stack = []   # (ours, taking, taken_any)
    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r'#ifndef (\w+)', s)
        if m and m.group(1) in vals and i + 2 < len(lines) and lines[i + 2].strip() == '#endif':
            i += 3
            continue
        active = all(t for _, t, _ in stack)
        if s.startswith('#if ') or s.startswith('#ifdef') or s.startswith('#ifndef'):
            v = cexpr(s[3:], vals) if s.startswith('#if ') else None
            if v is None:
                stack.append((False, True, True))
                if active:
                    out.append(ln)
            else:
                stack.append((True, bool(v), bool(v)))
            i += 1
            continue
        if s.startswith('#elif') and stack and stack[-1][0]:
            _, _, taken = stack[-1]
            v = cexpr(s[5:], vals)
            if v is None:
                raise SystemExit(f'{path}:{i + 1}: #elif mixes unknown macros')
            stack[-1] = (True, (not taken) and bool(v), taken or bool(v))
            i += 1
            continue
        if s.startswith('#else') and stack and stack[-1][0]:
            _, _, taken = stack[-1]
            stack[-1] = (True, not taken, True)
            i += 1
            continue
        if s.startswith('#endif') and stack:
            ours, _, _ = stack.pop()
            if not ours and all(t for _, t, _ in stack):
                out.append(ln)
            i += 1
            continue
        if active:
            for k, v in vals.items():
                ln = re.sub(r'\b%s\b' % k, str(v), ln)
            out.append(ln)
        i += 1
    open(path, 'w').write('\n'.join(out))


if __name__ == '__main__':
    main()
