set -e
TAG=r03-v10 bash tools/gpu.sh pmc:lane10 pmc:lane10l pmc:n256 pmc:n256l
BENOR_NO_MFMA=1 TAG=r03-v10-lane bash tools/gpu.sh pmc:lane10 pmc:lane10l
