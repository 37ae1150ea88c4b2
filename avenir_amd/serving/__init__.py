"""avenir_amd.serving"""
