"""Applications built on the framework (reference ppe_main_ddp.py)."""
