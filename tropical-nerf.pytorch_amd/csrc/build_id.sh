#!/bin/sh
# Build id of libtropical_hip.so: a hash of the sources it is built from
# (include/*.h, csrc/*.hip *.h *.cpp and the Makefile), compiled into the
# library as tnp_build_id().  tropical/_hip.py recomputes it from the tree
# it loads the library from and refuses a library built from other sources
# (tropical/_buildid.py is the same rule in Python).
cd "$(dirname "$0")" || exit 1
{
  for f in ../../include/*.h; do printf 'include/%s %s\n' "${f##*/}" "$(sha256sum < "$f" | cut -c1-64)"; done
  for f in *.hip *.h *.cpp Makefile; do printf 'csrc/%s %s\n' "$f" "$(sha256sum < "$f" | cut -c1-64)"; done
} | LC_ALL=C sort | sha256sum | cut -c1-16
