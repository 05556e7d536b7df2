# A/B variant: only the test kernel's half of scripts/patch_lv_pipe.py (grid row in LDS).
import os
os.environ['LV_PART'] = 'grid'
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'patch_lv_pipe.py')).read())
