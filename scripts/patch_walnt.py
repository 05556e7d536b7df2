# Diagnostic variant (scripts/build_variant.sh): the WAL segment kernel's scratch entries written with non-temporal stores
s = open('decode.hip').read()
old = '''                dst[i] = (p - start) | (kl < kWalKlEsc ? kl : kWalKlEsc) << kWalPosBits;'''
assert old in s
s = s.replace(old, '''                __builtin_nontemporal_store((p - start) | (kl < kWalKlEsc ? kl : kWalKlEsc) << kWalPosBits, &dst[i]);''')
open('decode.hip', 'w').write(s)
