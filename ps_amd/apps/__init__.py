"""Reference demo applications (CTR.java, Mnist.java, CnnMnist.java) on ps_amd."""
