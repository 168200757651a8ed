import re
import sys
R=sys.argv[1].rstrip('/')+'/'
def edit(p, pairs):
    s=open(R+p).read()
    for old,new in pairs:
        assert s.count(old)==1,(p,old[:70],s.count(old))
        s=s.replace(old,new)
    open(R+p,'w').write(s)
edit('trajopt-1_amd/csrc/layout.hpp',[(
'''  int chm_hbm;
''','''  int chm_hbm;
  // wide blocks whose chain matrices fit the LDS next to the factor (2 sN sD^2
  // doubles <= kWideChmLds: the waypoint-pair solve of JointAccEqCost problems,
  // 15 blocks of 14 dofs): M, N in the LDS scratch like narrow blocks, read by the
  // wide chain through LDS-typed pointers instead of HBM round trips
  int wide_lds;
'''),(
'''constexpr long long kLdsBudgetGenBytes = 146 * 1024;
''','''constexpr long long kLdsBudgetGenBytes = 146 * 1024;
// the most doubles of wide-block chain matrices kept in LDS (Layout::wide_lds)
constexpr long long kWideChmLds = 6144;
''')])
edit('trajopt-1_amd/csrc/thip_api.hip',[(
'''  sizes[A_CHM] = (L.wide || L.chm_hbm) ? 2 * sNDD : 1;''','''  L.wide_lds = (L.wide && 2 * sNDD <= kWideChmLds) ? 1 : 0;
  sizes[A_CHM] = ((L.wide && !L.wide_lds) || L.chm_hbm) ? 2 * sNDD : 1;'''),(
'''  const size_t lds_d = std::max<size_t>({ (size_t)((L.wide || L.chm_hbm) ? 0 : 2 * sNDD),''','''  const size_t lds_d = std::max<size_t>({ (size_t)(((L.wide && !L.wide_lds) || L.chm_hbm) ? 0 : 2 * sNDD),''')])
edit('trajopt-1_amd/csrc/sqp_kernel.hip',[(
'''  sv.M = (L.wide || L.chm_hbm) ? wsb + L.doff[A_CHM] : dyn;''','''  sv.M = ((L.wide && !L.wide_lds) || L.chm_hbm) ? wsb + L.doff[A_CHM] : dyn;'''),(
'''__device__ __noinline__ void block_chain_wide(const double* Gp, const double* cvp, double* outp, int t0, int nsteps,
                                              int dir, bool store_first, int D, int lane)
{
  const gbl_f64* G = gbl(Gp);  // HBM (Layout::wide)
''','''template <typename GP>
__device__ __noinline__ void block_chain_wide(GP G, const double* cvp, double* outp, int t0, int nsteps, int dir,
                                              bool store_first, int D, int lane)
{
  // G: HBM (Layout::wide), or LDS (Layout::wide_lds)
'''),(
'''  if (wide)
    block_chain_wide(G, cv, out, t0, nsteps, dir, store_first, D, lane);
  else if (chm_hbm)''','''  if (wide)
  {
    if (chm_hbm)  // (wide: chm_hbm carries "not Layout::wide_lds")
      block_chain_wide(gbl(G), cv, out, t0, nsteps, dir, store_first, D, lane);
    else
      block_chain_wide(lds(G), cv, out, t0, nsteps, dir, store_first, D, lane);
  }
  else if (chm_hbm)'''),
])
s=open(R+'trajopt-1_amd/csrc/sqp_kernel.hip').read()
n=s.count('L.sD, c.lane, L.wide, L.chm_hbm);')
assert n==4, n
s=s.replace('L.sD, c.lane, L.wide, L.chm_hbm);','L.sD, c.lane, L.wide, L.chm_hbm || (L.wide && !L.wide_lds));')
old='''__device__ __noinline__ void twisted_middle_wide(const Ctx& c, const Solver& sv, const double* LIp, double* CVp,
                                                double* YVp)
{
  // solve blocks (Layout::grp: a waypoint pair), one branch
  const int D = c.L.sD, DD = D * D, m = c.L.tw_mid, N = c.L.sNb, i = c.lane;
  const lds_f64* LI = lds(LIp);
  const gbl_f64* M = gbl(sv.M);  // HBM (Layout::wide)
  const gbl_f64* Mb = gbl(sv.Nb);'''
new='''template <typename MP>
__device__ __noinline__ void twisted_middle_wide(const Ctx& c, MP M, MP Mb, const double* LIp, double* CVp,
                                                double* YVp)
{
  // solve blocks (Layout::grp: a waypoint pair), one branch; M, Mb in HBM
  // (Layout::wide) or LDS (Layout::wide_lds)
  const int D = c.L.sD, DD = D * D, m = c.L.tw_mid, N = c.L.sNb, i = c.lane;
  const lds_f64* LI = lds(LIp);'''
assert s.count(old)==1; s=s.replace(old,new)
old='''  if (c.L.wide)
    twisted_middle_wide(c, sv, LIp, CVp, const_cast<double*>(YVp));'''
new='''  if (c.L.wide && c.L.wide_lds)
    twisted_middle_wide(c, lds(static_cast<const double*>(sv.M)), lds(static_cast<const double*>(sv.Nb)), LIp, CVp,
                        const_cast<double*>(YVp));
  else if (c.L.wide)
    twisted_middle_wide(c, gbl(static_cast<const double*>(sv.M)), gbl(static_cast<const double*>(sv.Nb)), LIp, CVp,
                        const_cast<double*>(YVp));'''
assert s.count(old)==1; s=s.replace(old,new)
open(R+'trajopt-1_amd/csrc/sqp_kernel.hip','w').write(s)
print('wide_lds applied')
