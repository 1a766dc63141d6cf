import sys, os
sys.path.insert(0, os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'bevy-hikari_amd'))
from hikari_amd import HikariRenderer
r = HikariRenderer(0)
print("rcp mismatches", r.selftest_rcp(0, 0x80000000), flush=True)
print("in range [2^-125, 2^125]:", r.selftest_rcp(0x01000000, 0x7E000001), flush=True)
