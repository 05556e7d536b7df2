# Diagnostic library variant: copies go-lsm_amd/csrc to a scratch dir, applies
# a python patch script ($1, edits files in the cwd) and links ab/$2.so.
# Never the product library.
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
W=$(mktemp -d /tmp/var.XXXX)
cp -r $ROOT/go-lsm_amd/csrc $W/
(cd $W/csrc && python3 $1)
pids=""
for f in api decode encode merge; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$W/csrc -c $W/csrc/$f.hip -o $W/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/ab/$2.so $W/*.o
rm -rf $W
echo built ab/$2.so
