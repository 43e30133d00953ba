import sys, os, numpy as np
sys.path.insert(0,'dsp-slam-rgbd_amd'); sys.path.insert(0,'.')
import synthetic as S
from deep_sdf.workspace import decoder_from_state
from reconstruct.optimizer import Optimizer
from reconstruct.utils import ForceKeyErrorDict
dec=decoder_from_state(S.make_decoder(1234),S.DEFAULT_SPECS)
opt=Optimizer(dec,ForceKeyErrorDict(data_type="KITTI",optimizer=S.KITTI_OPTIM))
objs=[S.kitti_object(i) for i in range(16)]
res,tr=opt.reconstruct_objects([(o.t_cam_obj,o.pts,o.rays,o.depth,None) for o in objs],trace=True)
for i,(r,t) in enumerate(zip(res,tr)):
    print(i,r['is_good'],r['fail_reason'],r['iters_done'],'loss',r['loss'],'K',t['k'].tolist(),'nv',t['n_valid'].tolist())
r1=opt.reconstruct_object(objs[1].t_cam_obj,objs[1].pts,objs[1].rays,objs[1].depth)
print('single obj1',r1['is_good'],r1['loss'])
