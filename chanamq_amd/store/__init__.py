"""chanamq_amd.store"""
