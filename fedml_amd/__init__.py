"""fedml_amd — MI355X-native server-side federated aggregation for FedML."""
__version__ = "0.1.0"
