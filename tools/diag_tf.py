"""Teacher-forced GPU step vs golden, per component (diagnostic)."""
import sys, numpy as np
sys.path.insert(0, 'dsp-slam-rgbd_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import synthetic as S
from conftest import golden, make_cfg
from deep_sdf.workspace import decoder_from_state
from reconstruct.optimizer import Optimizer
dec = decoder_from_state(S.make_decoder(1234), S.DEFAULT_SPECS)
for name, optim, dt in [("kitti0", S.KITTI_OPTIM, "KITTI"), ("redwood0", S.REDWOOD_OPTIM, "Redwood")]:
    f = golden(f"f4_traj_{name}.npz")
    one = dict(optim, joint_optim=dict(optim["joint_optim"], num_iterations=1))
    opt = Optimizer(dec, make_cfg(one, dt))
    n = int(f["n_iters_run"])
    objs = [(f["it_t_obj_cam"][e], f["obj_pts"], f["obj_rays"], f["obj_depth"], f["it_z"][e]) for e in range(n)]
    res, tr = opt.reconstruct_objects(objs, trace=True, pose_is_obj_cam=True)
    for e in range(n):
        t = tr[e]
        print(name, e, "sdf", t["sdf_loss"][0], f["it_sdf_loss"][e], "rel", (t["sdf_loss"][0]-f["it_sdf_loss"][e])/f["it_sdf_loss"][e],
              "ren", t["render_loss"][0], f["it_render_loss"][e], "rel", (t["render_loss"][0]-f["it_render_loss"][e])/f["it_render_loss"][e],
              "K", t["k"][0], f["it_k"][e], "nv", t["n_valid"][0], f["it_n_valid"][e])
