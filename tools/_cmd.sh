set -e
tools/ab.sh "base ilp al64 prio" 2 --fpl 16 --spp 64 --modes 1,3,4
