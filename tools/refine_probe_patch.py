"""Timing-only variant of k_pnp_refine (tooling): per-stage wall-clock stamps (compaction, DLT
accumulation, DLT Jacobi, initial pose, LM) written into the frame's last RANSAC model slots.
    python tools/refine_probe_patch.py forest-slam_amd/csrc/pose.hip exp/pose_probe.hip
    python tools/build_variant.py probe exp/pose_probe.hip:pose.hip
    FVO_LIB=exp/libfvo_probe.so python tools/refine_probe.py [--hd]      (on the GPU box)"""
import sys
s = open(sys.argv[1]).read()
def rep(a, b):
    global s
    assert s.count(a) == 1, a
    s = s.replace(a, b)
rep('''  int ninl;
  int flag;
};''', '''  int ninl;
  int flag;
  double ts[8];
};''')
if 'sh.llp[k] = t;' in s:
    rep('''    if (lane == 0) sh.llp[k] = t;  // in LDS: the SVD below runs beside no register copy of it
  }
  __syncthreads();''', '''    if (lane == 0) sh.llp[k] = t;  // in LDS: the SVD below runs beside no register copy of it
  }
  __syncthreads();
  if (lane == 0) sh.ts[2] = (double)wall_clock64();''')
    import re
    m = re.search(r'  if \(!planar\) dlt12_null\([^\n]*\n', s)
    s = s[:m.end()] + '  if (lane == 0) sh.ts[3] = (double)wall_clock64();\n' + s[m.end():]
rep('''  // ---- Levenberg-Marquardt (CvLevMarq semantics)''', '''  if (lane == 0) sh.ts[4] = (double)wall_clock64();
  // ---- Levenberg-Marquardt (CvLevMarq semantics)''')
rep('''  if (lane == 0) sh.flag = 1;
  __syncthreads();
}''', '''  if (lane == 0) { sh.flag = 1; sh.ts[5] = (double)wall_clock64(); sh.ts[6] = iters; }
  __syncthreads();
}''')
rep('''  const int b = blockIdx.x, lane = threadIdx.x;
  const PnpState st = state[b];''', '''  const int b = blockIdx.x, lane = threadIdx.x;
  if (lane == 0) { sh.ts[0] = (double)wall_clock64(); for (int i = 1; i < 8; ++i) sh.ts[i] = 0; }
  const PnpState st = state[b];''')
rep('''  lm_refine(sh, K, Pc, Qc, ninl, mn_buf + (int64_t)b * cap * 2);''', '''  if (lane == 0) sh.ts[1] = (double)wall_clock64();
  lm_refine(sh, K, Pc, Qc, ninl, mn_buf + (int64_t)b * cap * 2);''')
rep('''    Tout[12] = 0; Tout[13] = 0; Tout[14] = 0; Tout[15] = 1;
    status[b] = 1;''', '''    Tout[12] = 0; Tout[13] = 0; Tout[14] = 0; Tout[15] = 1;
    status[b] = 1;
    sh.ts[7] = (double)wall_clock64();
    double* pr = const_cast<double*>(model) + ((int64_t)b * maxIters + maxIters - 2) * 6;
    for (int i = 0; i < 8; ++i) pr[i] = sh.ts[i];
    pr[8] = sh.ninl;''')
open(sys.argv[2], 'w').write(s)
