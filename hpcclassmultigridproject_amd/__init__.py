"""MI355X-native geometric multigrid for 2-D advection-diffusion (Crank-Nicolson).

Drop-in for the hot path of soniareilly/HPCClassMultigridProject: the V-cycle
(multigrid.cpp:17-120) and its stencil ops (gs.cpp), implemented as CDNA4 HIP
kernels in libmgx.so behind the C ABI of include/mgx.h.
"""
from . import gs
from ._lib import MGXError, Options, default_options, lib
from .multigrid import (Multigrid, default_maxlvl, init_problem, init_problem_rows,
                        timestepper, write_uT)

__all__ = ["gs", "MGXError", "Options", "default_options", "lib", "Multigrid",
           "default_maxlvl", "init_problem", "init_problem_rows", "timestepper", "write_uT"]
