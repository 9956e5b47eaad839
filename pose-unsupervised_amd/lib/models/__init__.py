"""PoseResNet family on MI355X HIP kernels (drop-in for the reference lib/models)."""
import models.pose_resnet  # noqa: F401
import models.multiview_pose_resnet  # noqa: F401
