"""avenir_amd.ops"""
