"""Drivers of the reference's experiments/ directory (sampling loops, MCEM, UCI data loading) on
the MI355X engine: experiments/utils_training.py, utils_training_demo.py, utils_dataset.py and
datasets.py, with the same function names and signatures."""
