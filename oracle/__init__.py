"""ORACLE — CPU restatement of the reference's PCG hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / the CPU baseline — never as a product
path.  The product (mlff-preconditioner_amd/, libmlffpcg.so) never imports it.

Every function cites the reference file:line it restates (paths relative to the
reference tree, bluecher31/mlff-preconditioner):

  pcg.cg_legacy             scipy 1.7.3 scipy.sparse.linalg.cg (CGREVCOM + python wrapper)
                            as called at src/sGDML/sgdml/solvers/iterative_solver.py:995-1005
  precon.pivoted_cholesky   src/sGDML/sgdml/solvers/incomplete_cholesky.py:24-93
  precon.woodbury_panel     src/sGDML/sgdml/solvers/iterative_cholesky.py:115-150
  precon.nystrom_panel      src/sGDML/sgdml/solvers/iterative_solver.py:95-322 (variant 0)
                            src/sGDML/sgdml/solvers/iterative_solver.py:326-381 (variant 1, _sb)
  precon.cho_factor_stable  src/sGDML/sgdml/solvers/iterative_solver.py:555-583
  precon.lev_scores         src/sGDML/sgdml/solvers/iterative_solver.py:447-552
  precon.svd_panel          src/sGDML/sgdml/solvers/iterative_solver.py:1177-1329
  sgdml.descriptors         src/sGDML/sgdml/utils/desc.py:80-358
  sgdml.assemble_kernel     src/sGDML/sgdml/train.py:81-236, 1121-1308
  rbf.rbf_kernel            src/tools/utils.py:173-187 (sklearn RBF)
  rot.rule_of_thumb         src/tools/plot_data.py:677-734, 1254-1258

Pinning: tests/golden/make_golden.py ran the reference itself (imported from
/root/reference in the development container) and committed its outputs as
tests/golden/*.npz; tests/test_oracle_golden.py checks this restatement against
them.  The scipy 1.7.3 CG recurrence is third-party (scipy==1.7.3 pinned in the
reference's environment.yml:11, not installed here); it is restated from the
published CGREVCOM template and the 1.7.3 python wrapper, and cross-checked by
an independent reverse-communication transliteration in make_golden.py.
"""
