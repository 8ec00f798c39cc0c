# rocprofv3 evidence for round 4: tools/profile.sh (single, many, packed, stress, config4) + profile_aux.sh
set -o pipefail
bash tools/profile.sh r04 || { echo "profile.sh failed"; exit 1; }
bash tools/profile_aux.sh r04 || { echo "profile_aux.sh failed"; exit 1; }
echo profiles done
