cd "$GRAFT_REPO_ROOT" || exit 1
for v in base sig1 sig2; do
  if [ "$v" = base ]; then lib=""; else lib="MDQT_LIB=expt/$v/lib/libmdqt.so"; fi
  echo "== $v"; timeout -k 10 120 env $lib python3 tools/sig_probe.py || exit 1
done
