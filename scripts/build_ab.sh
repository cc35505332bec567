# Build an A/B variant of libsrf.so with extra flags on some sources:
#   bash scripts/build_ab.sh NAME "A.hip B.hip" "-DFLAG=1"
set -e
NAME=$1; SRC=$2; FLAGS=$3
ROOT=$(cd $(dirname $0)/.. && pwd)
C=$ROOT/srf_amd/csrc
mkdir -p $ROOT/ab $ROOT/build/ab_$NAME
objs=""
for f in $C/*.hip $C/*.cpp; do
  b=$(basename $f); o=$ROOT/build/csrc/${b%.*}.o
  if [[ " $SRC " == *" $b "* ]]; then
    o=$ROOT/build/ab_$NAME/${b%.*}.o
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -munsafe-fp-atomics $FLAGS -c $f -o $o
  fi
  objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $ROOT/ab/$NAME.so $objs
echo built ab/$NAME.so
