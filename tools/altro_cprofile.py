import cProfile, pstats, sys, os, io, logging
sys.path[:0] = ["dcol-trajectory-optimization_amd", "."]
from altro import solve, systems
logging.getLogger("altro").setLevel(logging.WARNING)
params, X, U = systems.initialize("quadrotor")
solve(params, X, U, verbose=False)
params, X, U = systems.initialize("quadrotor")
pr = cProfile.Profile()
pr.enable()
r = solve(params, X, U, verbose=False)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
print(s.getvalue()[:6000])
print("ms/iter", r.ms_per_iter)
