#!/bin/bash
# scripts/k1_pmc_flags.sh -- dynamic instruction counts of K1 under the diag
# build's switches (MIJ_K1_FLAGS): one PMC pass per flag set.
# FLAGS="0 1 ..." MODE=encode|dct KRE=<kernel regex>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
[ -f jpeg-encoder-decoder_amd/libmijpeg_diag.so ] || { echo "make -C jpeg-encoder-decoder_amd diag first"; exit 1; }
for f in ${FLAGS:-0}; do
  echo "flags=$f"
  MIJ_LIB=$PWD/jpeg-encoder-decoder_amd/libmijpeg_diag.so MIJ_K1_FLAGS=$f TAG=_f$f bash scripts/k1_pmc_quick.sh || exit 1
done
