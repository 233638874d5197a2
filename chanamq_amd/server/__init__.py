"""chanamq_amd.server"""
