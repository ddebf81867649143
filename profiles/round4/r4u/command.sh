# the final tree, exactly the driver's commands
bash scripts/gpu_run.sh r4u "driver_pytest:1200:python -m pytest tests -m gpu -x -q" smoke bench
