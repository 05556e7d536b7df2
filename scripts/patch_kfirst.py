# Diagnostic variant (scripts/build_variant.sh): lsm_build_sst_views_gather queues the key copy before the data-region copy
s = open('encode.hip').read()
old = '''            vregion();
            if (rc == 0) {
                const int g = gather_keys_launch(views->bytes, kg->kd, kg->vd, kg->idx, kg->d_nout, kg->nmax,
                                                 kg->keys, d_koff, d_voff, kg->ws, kg->ws_bytes, rs);
                if (g && rc == 0) rc = g;
            }'''
assert old in s
s = s.replace(old, '''            {
                const int g = gather_keys_launch(views->bytes, kg->kd, kg->vd, kg->idx, kg->d_nout, kg->nmax,
                                                 kg->keys, d_koff, d_voff, kg->ws, kg->ws_bytes, rs);
                if (g && rc == 0) rc = g;
            }
            if (rc == 0) vregion();''')
open('encode.hip', 'w').write(s)
