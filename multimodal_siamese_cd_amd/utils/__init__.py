"""Reference-compatible `utils` package: networks, loss_functions, experiment_manager, parsers, datasets."""
