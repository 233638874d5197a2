"""chanamq_amd.broker"""
