# A/B variant: the level search's may-bit written by classify for every probe (1 for a
# candidate whose filter the test will read), the test writing only the 0s of failed
# candidates (fewer scattered byte stores).
s = open('encode.hip').read()
old = '''        if (!test) {
            may[i] = 0;
            continue;
        }
        cand[p] = idx;'''
assert old in s
s = s.replace(old, '''        may[i] = test ? 1 : 0;  // the test clears a candidate whose bit is 0
        if (!test) continue;
        cand[p] = idx;''')
old = '''        else may[k_begin + id] = (uint8_t)r;'''
assert old in s
s = s.replace(old, '''        else if (!r) may[k_begin + id] = 0;''')
open('encode.hip', 'w').write(s)
print('ok mayonce')
