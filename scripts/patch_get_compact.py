# A/B variant: applies scripts/patch_get_compact.diff (the Get kernel working only on
# probes whose may-bit is set, compacted per wave through LDS) to the csrc copy.
import os, subprocess
d = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'patch_get_compact.diff')
subprocess.run(['patch', '-p3', '-i', d], check=True)
print('ok getc')
