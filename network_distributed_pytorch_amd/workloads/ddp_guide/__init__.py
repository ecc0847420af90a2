"""See ddp_init.py / run_script.py."""
