"""CPU oracle for the batched NMPC hot path — TEST INFRASTRUCTURE ONLY.

This package restates, on the CPU in fp64, what the reference computes on its hot path
(`AcadosOcpSolver.solve()` inside the closed loops of
`src/force_model/controller.py:25-54` and `src/jerk_model/controller.py:26-56`).

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import,
call or link anything under `oracle/`, and only as the checker / reported CPU baseline.
The product path (`drone_attitude_control_amd`) never imports it and fails loudly when
its HIP library is missing.

Parity status:
  * constants and the reference trajectory are PINNED against fixtures generated from the
    reference's own importable modules (tests/golden/make_golden.py: params.py,
    generate_trajectory.py);
  * the QP solve is "parity unpinned" versus acados (acados_template / casadi / HPIPM are not
    installed and cannot be fetched; the reference ships no tests or recorded outputs).
    The oracle instead certifies every QP solution by its KKT conditions (a strictly convex
    QP has exactly one KKT point), computed by a dense condensed interior-point method plus
    an active-set polish — a formulation independent of the stage-wise Riccati recursion
    the GPU kernel uses.

Modules:
  params       — DroneData / ExperimentParameters constants (params.py:10-122)
  trajectory   — gen_circle_traj (generate_trajectory.py:7-28)
  models       — controller models + discretisation (force/jerk dynamics.py, ocp.py) and the
                 synthetic quad13 model used for the headline metric dimensions
  qp           — condensed dense QP, Mehrotra IPM, active-set polish, KKT certificate
  closed_loop  — follow_trajectory restatements, converters, plant simulators, calc_aed
  c/           — plain-C fp64 Riccati interior-point batch solver (CPU baseline "port")
"""
