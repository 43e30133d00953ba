set -u
bash tools/ab_lib.sh sA dsp-slam-rgbd_amd/csrc/libdsr.so dsp-slam-rgbd_amd/csrc/exp_maxilp.so || exit $?
bash tools/ab_lib.sh sB dsp-slam-rgbd_amd/csrc/libdsr.so dsp-slam-rgbd_amd/csrc/exp_maxmc.so || exit $?
