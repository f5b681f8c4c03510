cd $GRAFT_REPO_ROOT && bash tools/profile_round.sh r02 && python3 tools/pmc_summary.py gpurun_out/r02/pmc nlse3d_512 16 134217728 gpurun_out/r02/pmc_nlse3d_512.json k_tail 0.2857
