# Diagnostic library from a git revision ($1) of go-lsm_amd/csrc and the C ABI
# header, linked as ab/$2.so (for A/B against the working tree's library).
# Never the product library.
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
W=$(mktemp -d /tmp/rev.XXXX)
(cd $ROOT && git archive $1 go-lsm_amd/csrc include | tar -x -C $W)
pids=""
for f in api decode encode merge; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$W/include -I$W/go-lsm_amd/csrc -c $W/go-lsm_amd/csrc/$f.hip -o $W/$f.o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
mkdir -p $ROOT/ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $ROOT/ab/$2.so $W/*.o
rm -rf $W
echo built ab/$2.so from $1
