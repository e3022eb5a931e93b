import sys, numpy as np
sys.path.insert(0,'pfilter-noetic_amd'); sys.path.insert(0,'pfilter-noetic_amd/synth'); sys.path.insert(0,'oracle')
import pfilter_amd as pa, pfsynth, pfref
x = pfsynth.Sequence('S32', n_frames=2).frame(1)
g,u = pfref.ground_seg(x[:, :3]); U = x[u]
dc = pa.Dcvc(max_points=100000)
for k in range(3):
    i, l = dc.run(U); print("call", k, len(i), "clusters", l.max())
dc.reset(); i, l = dc.run(U); print("after reset", len(i))
for ff in (True, False):
    i, l = pfref.dcvc(U, first_frame=ff, components=True); print("oracle first", ff, len(i), "clusters", l.max())
dc2 = pa.Dcvc(max_points=100000); i,l = dc2.run(U[:100]); i, l = dc2.run(U); print("warm", len(i))
import ctypes
L = pa.lib(); L.pf_dcvc_debug.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
d3 = pa.Dcvc(max_points=100000)
for k in range(2):
    d3.run(U); o = np.zeros(8); L.pf_dcvc_debug(d3._h, o.ctypes.data); print("debug", k, o.tolist())
